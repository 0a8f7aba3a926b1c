#!/bin/bash
# igemmh numerics + per-GEMM timing of igemmh vs igemm3 for the conv GEMMs it serves (B=128)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k igemmh \
  > gpurun_out/h_tests.log 2>&1
rc=$?; tail -25 gpurun_out/h_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u benchmarks/bench_kernels.py --batch 128 --reps 10 --out gpurun_out/tuned_h.json \
  > gpurun_out/tune_h.log 2>&1
rc=$?; cut -c1-250 gpurun_out/tune_h.log; exit $rc
