#!/bin/bash
# round 5: 28x28 and 256x256 fp16 re-tunes (only their kept keys, on top of the shipped table) vs the shipped table, interleaved
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
T=benchmarks/tuned_tables/tuned_eager28_alt1_r5.json
for i in 1 2 3; do
  r=$(timeout -k 10 120 python3 bench.py --output_size 28 --c_dim 1 --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "28 shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 120 python3 bench.py --output_size 28 --c_dim 1 --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "28 retuned :: $r"
done | tee gpurun_out/ab_t28_alt1.txt
T=benchmarks/tuned_tables/tuned_eager256_fp16_p2_r5.json
for i in 1 2; do
  r=$(timeout -k 10 300 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | js) || exit 1; echo "256 shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 300 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | js) || exit 1; echo "256 retuned :: $r"
done | tee gpurun_out/ab_t256_p2.txt
