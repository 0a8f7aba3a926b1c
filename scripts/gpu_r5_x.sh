#!/bin/bash
# round 5: linear fwd / wgrad with all loads in flight -- tests (kernel + whole-step parity), A/B vs ab_old/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_kernels.py \
  tests/test_hip_engine.py -k "linear or matches_reference or stagewise" > gpurun_out/r5x_tests.log 2>&1 || { tail -40 gpurun_out/r5x_tests.log; exit 1; }
tail -2 gpurun_out/r5x_tests.log
for i in 1 2 3 4; do
  r=$(timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | grep '^{' | cut -c75-130) || exit 1; echo "new :: $r"
  r=$(cd ab_old && timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | grep '^{' | cut -c75-130) || exit 1; echo "old :: $r"
done | tee gpurun_out/ab_linear_inflight.txt
