#!/bin/bash
# Bench every BASELINE config family on one MI355X (synthetic data, random init).
mkdir -p gpurun_out
out=gpurun_out/bench_configs.jsonl; : > $out
run() {  # run <timeout> <args...>
  local t=$1; shift
  timeout -k 10 "$t" python bench.py "$@" > gpurun_out/bc.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; tail -20 gpurun_out/bc.log; exit $rc; fi
  tail -1 gpurun_out/bc.log >> $out; tail -1 gpurun_out/bc.log | cut -c1-220
}
run 300 --steps 200 --warmup 20
run 300 --steps 50 --warmup 10 --dtype fp16
run 300 --steps 20 --warmup 5 --dtype fp32
run 300 --steps 30 --warmup 5 --output_size 28 --c_dim 1
run 300 --steps 20 --warmup 5 --output_size 128
run 600 --steps 10 --warmup 3 --output_size 256 --batch_size 512 --dtype fp16
