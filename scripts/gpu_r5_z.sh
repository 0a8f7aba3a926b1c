#!/bin/bash
# round 5: 128x128 bf16 in-situ re-tune vs the shipped table, 4 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3 4; do
  r=$(timeout -k 10 200 python3 bench.py --output_size 128 --steps 40 --warmup 5 2>/dev/null | js) || exit 1; echo "shipped :: $r"
  r=$(DCGAN_TUNED_PATH=benchmarks/tuned_tables/tuned_t128_r5.json timeout -k 10 200 python3 bench.py --output_size 128 --steps 40 --warmup 5 2>/dev/null | js) || exit 1; echo "retuned :: $r"
done | tee gpurun_out/ab_t128.txt
