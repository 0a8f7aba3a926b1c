#!/bin/bash
# round 5: remaining schedule knobs under the re-tuned table (nconv persistent-grid cap, G-chain-first issue), interleaved
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  for v in "X=0" "DCGAN_NCONV_CAP=256" "DCGAN_NCONV_CAP=1024" "DCGAN_G_FIRST=3" "DCGAN_G_FIRST=8"; do
    r=$(env $v timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "$v :: $r"
  done
done | tee gpurun_out/ab_knobs_retuned_r5.txt
