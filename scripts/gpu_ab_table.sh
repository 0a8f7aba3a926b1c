#!/bin/bash
# A/B of two tile tables on the headline bench: $1 = candidate table (DCGAN_TUNED_PATH) vs the shipped one, x3
mkdir -p gpurun_out
for i in 1 2 3; do
  echo "[shipped]"; timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null | cut -c1-200 || exit 1
  echo "[$1]"; DCGAN_TUNED_PATH=$1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null | cut -c1-200 || exit 1
done | tee gpurun_out/ab_table.txt
