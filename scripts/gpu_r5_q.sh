#!/bin/bash
# round 5: tile table with wgrad5 (410) for the two 64-channel weight gradients vs the shipped table
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["kernels_per_step"])'; }
for i in 1 2 3 4; do for t in shipped tuned_w5c_r5 tuned_w5d_r5; do
  if [ $t = shipped ]; then r=$(timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || exit 1
  else r=$(DCGAN_TUNED_PATH=benchmarks/tuned_tables/$t.json timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null | js) || exit 1; fi
  echo "$t :: $r"
done; done | tee gpurun_out/ab_wgrad5_table2.txt
