#!/bin/bash
# round 5: tail timeline of the fused step (no profiler) for 0-3 G weight gradients on cs,
# then an interleaved bench A/B of DCGAN_GW_TAIL_ON_MAIN 1/2/3
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/tail_timeline_r5.txt; : > $out
for t in 2 1 3 0; do
  timeout -k 10 120 python3 -u benchmarks/study/tail_timeline.py --tail-on-main $t >> $out 2>&1 || exit $?
done
ab=gpurun_out/ab_gw_tail2_r5.txt; : > $ab
for r in 1 2 3; do
  for t in 2 1 3; do
    v=$(DCGAN_GW_TAIL_ON_MAIN=$t timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | grep '^{') || exit $?
    echo "round $r tail_on_main=$t $v" >> $ab
  done
done
cat $out; cut -c1-120 $ab
