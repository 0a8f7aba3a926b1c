#!/bin/bash
# A/B of engine variants: interleaved bench runs (env var toggles)
mkdir -p gpurun_out; : > gpurun_out/ab.log
for i in 1 2 3; do
  for v in "" "DCGAN_SERIAL_WGRAD=1"; do
    env $v timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/ab1.log 2>&1 || { tail gpurun_out/ab1.log; exit 1; }
    echo "[$v] $(tail -1 gpurun_out/ab1.log | cut -c1-160)" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
