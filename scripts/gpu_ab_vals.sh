#!/bin/bash
# A/B of an environment variable over several values on the headline bench, interleaved x3:
# $1 = VAR, $2 = "v1 v2 ...", remaining args -> bench.py
mkdir -p gpurun_out
var=$1; vals=$2; shift 2
for i in 1 2 3; do for f in $vals; do
  r=$(env $var=$f timeout -k 10 120 python bench.py --steps 200 --warmup 20 "$@" 2>/dev/null) || { echo "FAILED $var=$f"; exit 1; }
  echo "[$var=$f] $(echo "$r" | cut -c1-170)"
done; done | tee gpurun_out/ab_$var.txt
