#!/bin/bash
# round 5, call I: issue order of the G chain vs the D chain in the eager fused step (DCGAN_G_FIRST)
mkdir -p gpurun_out
out=gpurun_out/ab_g_first_r5i.txt; : > $out
val() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
  for k in 0 1 3 6 12; do
    r=$(DCGAN_G_FIRST=$k timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 2>/dev/null) || { echo "bench failed" >> $out; exit 1; }
    echo "G_FIRST=$k :: $(echo "$r" | val)" | tee -a $out
  done
done
