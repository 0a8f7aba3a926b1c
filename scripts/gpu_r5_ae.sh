#!/bin/bash
# round 5: G weight gradients on an idle stream beside both chains (DCGAN_GW_STREAM) vs behind
# the D chain, interleaved bench A/B
set -o pipefail
mkdir -p gpurun_out
ab=gpurun_out/ab_gw_stream_r5.txt; : > $ab
for r in 1 2; do
  for v in d:2 side:0 side:2 alt1:0 alt1:2 side:1; do
    s=${v%:*}; t=${v#*:}
    x=$(DCGAN_GW_STREAM=$s DCGAN_GW_TAIL_ON_MAIN=$t timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | grep '^{') || exit $?
    echo "round $r gw_stream=$s tail_on_main=$t $x" >> $ab
  done
done
cut -c1-110 $ab
