#!/bin/bash
# round 5: second 128x128 pass (sibling tiles) vs the shipped table, interleaved
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
T=benchmarks/tuned_tables/tuned_eager128_alt1_p2_r5.json
for i in 1 2 3 4; do
  r=$(timeout -k 10 200 python3 bench.py --output_size 128 --steps 60 --warmup 10 2>/dev/null | js) || exit 1; echo "128 shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 200 python3 bench.py --output_size 128 --steps 60 --warmup 10 2>/dev/null | js) || exit 1; echo "128 retuned :: $r"
done | tee gpurun_out/ab_t128_alt1_p2.txt
