#!/bin/bash
# igemm3 tile / pipeline-depth / split-K sweep for every conv GEMM of the 64x64 step at B=128
mkdir -p gpurun_out
timeout -k 10 900 python -u benchmarks/bench_kernels.py --batch 128 --reps 15 --out gpurun_out/tuned_b128.json \
  > gpurun_out/tune_b128.log 2>&1
rc=$?; cat gpurun_out/tune_b128.log | cut -c1-250; exit $rc
