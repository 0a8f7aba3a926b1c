#!/bin/bash
# round 5: 256x256 fp16 in-situ re-tune (2 entries) vs the shipped table, 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  r=$(timeout -k 10 200 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | js) || exit 1; echo "shipped :: $r"
  r=$(DCGAN_TUNED_PATH=benchmarks/tuned_tables/tuned_t256_r5.json timeout -k 10 200 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | js) || exit 1; echo "retuned :: $r"
done | tee gpurun_out/ab_t256.txt
