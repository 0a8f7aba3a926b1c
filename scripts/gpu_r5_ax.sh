#!/bin/bash
# round 5: D's weight gradients on the side stream (DCGAN_D_WGRAD_SIDE, study) -- bit-identity test + interleaved A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_hip_engine.py -m gpu -x -q --timeout 240 --timeout-method thread -k "placements" > gpurun_out/gpu_tests_dws_r5.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_dws_r5.log; [ $rc -eq 0 ] || exit $rc
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  for v in 0 1; do
    r=$(DCGAN_D_WGRAD_SIDE=$v timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "d_wgrad_side=$v :: $r"
  done
done | tee gpurun_out/ab_d_wgrad_side_r5.txt
