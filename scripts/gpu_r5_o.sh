#!/bin/bash
# round 5: split-K reduction with several slabs in flight (wgrad3 / wgrad5): tests, per-layer sweep,
# step A/B vs ab_old/ (same tree before the change; DCGAN_BN_FOLD=0 for both)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py \
  -k "wgrad5 or wgrad3_conv" > gpurun_out/r5o_tests.log 2>&1 || { tail -40 gpurun_out/r5o_tests.log; exit 1; }
tail -2 gpurun_out/r5o_tests.log
timeout -k 10 400 python3 -u benchmarks/bench_wgrad.py --batch 128 --size 64 --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_wgrad5_64c.txt
for i in 1 2 3 4; do
  r=$(DCGAN_BN_FOLD=0 timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | grep '^{') || exit 1
  echo "new :: $(echo "$r" | cut -c1-110)"
  r=$(cd ab_old && DCGAN_BN_FOLD=0 timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | grep '^{') || exit 1
  echo "old :: $(echo "$r" | cut -c1-110)"
done | tee gpurun_out/ab_splitk_unroll.txt
