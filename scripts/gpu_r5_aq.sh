#!/bin/bash
# round 5: g_h1's weight gradient on its own stream (the re-tuned g_h2 wgrad on alt1 runs long, 80 workgroups), interleaved
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  for p in aaaa aaas aaad aasa; do
    r=$(DCGAN_GW_PLACE=$p timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "$p :: $r"
  done
done | tee gpurun_out/ab_gw_place_h1_r5.txt
