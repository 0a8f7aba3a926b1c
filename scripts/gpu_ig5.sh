#!/bin/bash
# igemm5 study on one MI355X: error map, numerics, per-layer timing vs igemm3. A step that fails
# its asserts (rc 1) does not stop the next one; a fault / abort / time-out (any other rc) does.
mkdir -p gpurun_out
step() {  # step <timeout> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$log 2>&1
  local rc=$?
  grep -v amdgpu.ids gpurun_out/$log | tail -${TAILN:-40}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
step 120 ig5_diag.log python -u benchmarks/study/ig5_diag.py 4 16 128 256 400,401,402,403,411,412,413
step 420 ig5_tests.log python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k igemm5
TAILN=60 step 600 ig5_bench.log python -u benchmarks/bench_kernels.py --batch 128 --reps 10 --top 8 ${BENCH_ARGS}
