#!/bin/bash
# round 5: 64x64 re-tune under the alt1 weight-gradient placement vs the shipped table, interleaved
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
T=benchmarks/tuned_tables/tuned_eager64_alt1_r5.json
for i in 1 2 3 4 5; do
  r=$(timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "retuned :: $r"
done | tee gpurun_out/ab_t64_alt1.txt
