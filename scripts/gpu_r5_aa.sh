#!/bin/bash
# round 5: trailing G weight gradients on the main stream (DCGAN_GW_TAIL_ON_MAIN) after wgrad5
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3 4; do for n in 1 2 3; do
  v=$(DCGAN_GW_TAIL_ON_MAIN=$n timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || exit 1
  echo "DCGAN_GW_TAIL_ON_MAIN=$n :: $v"
done; done | tee gpurun_out/ab_gw_tail_r5.txt
