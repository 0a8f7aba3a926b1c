#!/bin/bash
# round 6: GPU suite on the current tree (all failures listed), smoke, old/new .so A/B
# (200/20 and driver form), kernel trace of the new tree
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r6b.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -8 gpurun_out/gpu_tests_r6b.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6b.log 2>&1 || exit $?
for i in 1 2 3; do
  for a in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    r=$(timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[new $a] ${r:0:110}"
    r=$(cd ab_old && timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[old $a] ${r:0:110}"
  done
done | tee gpurun_out/ab_nconv_epi_prefetch_r6.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r6b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6b -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_r6b.log 2>&1 || exit 1
exit $rc
