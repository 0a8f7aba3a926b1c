#!/bin/bash
# round 6: engine + kernel tests, 3-way A/B (tree / tree with DCGAN_STEP_OVERLAP=0 / ab_old baseline
# .so), kernel trace of the tree
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_engine.py tests/test_hip_kernels.py tests/test_hip_ddp.py -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r6c.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests_r6c.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for a in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    r=$(timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[new $a] ${r:70:40}"
    r=$(DCGAN_STEP_OVERLAP=0 timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[new-noov $a] ${r:70:40}"
    r=$(cd ab_old && timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[old $a] ${r:70:40}"
  done
done | tee gpurun_out/ab_r6c.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r6c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6c -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_r6c.log 2>&1 || exit 1
