#!/bin/bash
# round 6: nwgrad chunk-invariant addressing -- kernel + engine tests, A/B vs ab_old, step PMC table
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r6f.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests_r6f.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for a in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    r=$(timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[new $a] ${r:70:40}"
    r=$(cd ab_old && timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1; echo "[old $a] ${r:70:40}"
  done
done | tee gpurun_out/ab_nwgrad_r6.txt
OUT=step_pmc_r6.txt ./scripts/gpu_pmc_step.sh > /dev/null || exit 1
head -30 gpurun_out/step_pmc_r6.txt
