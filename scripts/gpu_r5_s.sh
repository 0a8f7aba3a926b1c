#!/bin/bash
# round 5: wgrad5 table entries for 128x128 (bf16) and 256x256 (fp16, bs 512) vs the shipped table
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["kernels_per_step"])'; }
T=benchmarks/tuned_tables/tuned_w5_128_256_r5.json
for i in 1 2 3; do
  r=$(timeout -k 10 120 python3 bench.py --output_size 128 --steps 30 --warmup 5 2>/dev/null | js) || exit 1; echo "128 shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 120 python3 bench.py --output_size 128 --steps 30 --warmup 5 2>/dev/null | js) || exit 1; echo "128 wgrad5 :: $r"
done | tee gpurun_out/ab_wgrad5_128.txt
for i in 1 2 3; do
  r=$(timeout -k 10 200 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | js) || exit 1; echo "256 shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 200 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | js) || exit 1; echo "256 wgrad5 :: $r"
done | tee gpurun_out/ab_wgrad5_256.txt
