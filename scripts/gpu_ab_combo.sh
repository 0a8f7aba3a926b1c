#!/bin/bash
# interleaved A/B of environment combinations on the headline bench: each arg is one combination,
# e.g. "DCGAN_A=1 DCGAN_B=0"; 4 rounds; output gpurun_out/ab_combo.txt; BENCH_ARGS: extra bench.py args
# (default --steps 200 --warmup 20)
mkdir -p gpurun_out
for i in 1 2 3 4; do for combo in "$@"; do
  r=$(env $combo timeout -k 10 120 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20} 2>/dev/null) || { echo "FAILED $combo"; exit 1; }
  echo "[$combo] $(echo "$r" | sed 's/"metric": "[^"]*", //' | cut -c1-60)"
done; done | tee gpurun_out/ab_combo.txt
