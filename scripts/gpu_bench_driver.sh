#!/bin/bash
# The driver's exact 1-GPU command (20 timed / 5 warmup) $1 times, then the 50/10 default $1 times,
# interleaved, on this one lease (OUT: summary file under gpurun_out/).
mkdir -p gpurun_out
out=gpurun_out/${OUT:-bench_driver.txt}
: > $out
for i in $(seq 1 ${1:-3}); do
  for a in "--steps 20 --warmup 5" "--steps 50 --warmup 10"; do
    r=$(timeout -k 10 180 python3 bench.py --gpus 1 $a 2>/dev/null) || { echo "bench failed: $a" >> $out; exit 1; }
    echo "$a :: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"])')" | tee -a $out
  done
done
