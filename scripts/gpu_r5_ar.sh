#!/bin/bash
# round 5: fused step vs the segmented DDP step over a one-rank RCCL group, interleaved, same steps
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  r=$(timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "fused :: $r"
  r=$(timeout -k 10 150 python3 bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "force_ddp :: $r"
  r=$(DCGAN_DDP_GW_ALT=2 timeout -k 10 150 python3 bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "force_ddp gw_alt=2 :: $r"
done | tee gpurun_out/ab_fused_vs_ddp_r5.txt
