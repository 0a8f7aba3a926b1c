#!/bin/bash
# interleaved A/B/C of values of one env switch on the headline bench: $1 = VAR, $2.. = values
# (3 rounds, 200/20 and the driver's 20/5), summary in gpurun_out/ab_<VAR>.txt
mkdir -p gpurun_out
var=$1; shift
for i in 1 2 3; do
  for a in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    for v in "$@"; do
      r=$(env $var=$v timeout -k 10 120 python bench.py $a 2>/dev/null) || exit 1
      echo "[$var=$v $a] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"])')"
    done
  done
done | tee gpurun_out/ab_$var.txt
