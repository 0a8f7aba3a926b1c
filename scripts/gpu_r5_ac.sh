#!/bin/bash
# round 5: 64x64 re-tune after the longest-phase-first dispatch vs the shipped table, 5 interleaved rounds (+ driver form)
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
T=benchmarks/tuned_tables/tuned_t64c_r5.json
for i in 1 2 3 4 5; do
  r=$(timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || exit 1; echo "shipped :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || exit 1; echo "retuned :: $r"
done | tee gpurun_out/ab_t64c.txt
for i in 1 2; do
  r=$(timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 2>/dev/null | js) || exit 1; echo "shipped 20/5 :: $r"
  r=$(DCGAN_TUNED_PATH=$T timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 2>/dev/null | js) || exit 1; echo "retuned 20/5 :: $r"
done | tee -a gpurun_out/ab_t64c.txt
