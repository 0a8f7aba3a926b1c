#!/bin/bash
# round 5 study: the D-chain / weight-gradient streams restricted to (32 - r) of every 32 CUs
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do for r in 0 2 4 8; do
  v=$(DCGAN_ALT_CU_RESERVE=$r timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || { echo "FAILED $r"; exit 1; }
  echo "DCGAN_ALT_CU_RESERVE=$r :: $v"
done; done | tee gpurun_out/ab_alt_cu_reserve.txt
