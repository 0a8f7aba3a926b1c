#!/bin/bash
# round 5: igemm3 longest-phase-first dispatch (DCGAN_IGEMM_LPT): kernel tests + engine parity with it on, A/B at 64 / 256
set -o pipefail
mkdir -p gpurun_out
DCGAN_IGEMM_LPT=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_kernels.py \
  tests/test_hip_engine.py -k "igemm or deconv or matches_reference or stagewise" > gpurun_out/r5ab_tests.log 2>&1 || { tail -40 gpurun_out/r5ab_tests.log; exit 1; }
tail -2 gpurun_out/r5ab_tests.log
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3 4; do for f in 0 1; do
  v=$(DCGAN_IGEMM_LPT=$f timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || exit 1
  echo "64 DCGAN_IGEMM_LPT=$f :: $v"
done; done | tee gpurun_out/ab_lpt.txt
for i in 1 2; do for f in 0 1; do
  v=$(DCGAN_IGEMM_LPT=$f timeout -k 10 200 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | js) || exit 1
  echo "256 DCGAN_IGEMM_LPT=$f :: $v"
done; done | tee -a gpurun_out/ab_lpt.txt
