#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
T=benchmarks/tuned_tables/tuned_eager64_alt1_x_r5.json
for i in 1 2 3 4; do
  r=$(timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "64 shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "64 retuned :: $r"
done | tee gpurun_out/ab_t64_alt1_x.txt
