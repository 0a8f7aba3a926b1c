#!/bin/bash
# 8-wave igemm3 tiles: numerics, then the per-GEMM sweep over every conv GEMM (B=128)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_kernels.py \
  -k "igemm3 or igemmh or fused_bn_backward" > gpurun_out/w8_tests.log 2>&1
rc=$?; tail -30 gpurun_out/w8_tests.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u benchmarks/bench_kernels.py --batch 128 --reps 10 --top 8 --cfgs 2 \
  --out gpurun_out/tuned_w8.json > gpurun_out/tune_w8.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/tune_w8.log | cut -c1-300; exit $rc
