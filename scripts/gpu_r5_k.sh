#!/bin/bash
# round 5: BN fold with the 16-lane-group reduction: bit-exactness + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_hip_kernels.py tests/test_hip_engine.py -k "bn_fold or bn_forward_backward" \
  > gpurun_out/r5k_tests.log 2>&1 || { tail -30 gpurun_out/r5k_tests.log; exit 1; }
tail -2 gpurun_out/r5k_tests.log
for i in 1 2 3 4; do for f in 0 64 256; do
  r=$(DCGAN_BN_FOLD=$f timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null) || { echo "FAILED $f"; exit 1; }
  echo "DCGAN_BN_FOLD=$f :: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["kernels_per_step"])')"
done; done | tee gpurun_out/ab_bn_fold2.txt
