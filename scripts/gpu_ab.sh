#!/bin/bash
# GPU tests, then A/B of engine variants: interleaved bench runs (env var toggles in $AB)
mkdir -p gpurun_out; : > gpurun_out/ab.log
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for i in 1 2 3; do
  for v in "X=0" "$1"; do
    env $v timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/ab1.log 2>&1 || { tail gpurun_out/ab1.log; exit 1; }
    echo "[$v] $(tail -1 gpurun_out/ab1.log | cut -c90-150)" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
