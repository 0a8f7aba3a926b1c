#!/bin/bash
# round 5: Adam(D) early on the D chain's stream -- bit-exactness + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_engine.py \
  -k "early_adam" > gpurun_out/r5w_tests.log 2>&1 || { tail -40 gpurun_out/r5w_tests.log; exit 1; }
tail -2 gpurun_out/r5w_tests.log
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3 4; do for f in 0 1; do
  v=$(DCGAN_ADAM_D_EARLY=$f timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || exit 1
  echo "DCGAN_ADAM_D_EARLY=$f :: $v"
done; done | tee gpurun_out/ab_adam_d_early.txt
