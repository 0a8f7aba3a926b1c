#!/bin/bash
# A/B of an environment switch on the headline bench: $1 = VAR, runs VAR=0 / VAR=1 alternately x3
mkdir -p gpurun_out
var=$1; shift
for i in 1 2 3; do for f in 0 1; do
  echo "[$var=$f]"; env $var=$f timeout -k 10 120 python bench.py --steps 200 --warmup 20 "$@" 2>/dev/null | cut -c1-200 || exit 1
done; done | tee gpurun_out/ab_$var.txt
