#!/bin/bash
# round 5: G weight-gradient placements again under the re-tuned table, interleaved
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  for p in aaaa ssss aaac daaa sasa; do
    r=$(DCGAN_GW_PLACE=$p timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "$p :: $r"
  done
done | tee gpurun_out/ab_gw_place_retuned_r5.txt
