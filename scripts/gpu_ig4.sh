#!/bin/bash
# igemm4 bring-up: its numerics tests, then per-layer tile timings (every step bounded; stop at the first failure)
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_hip_kernels.py -x -v -k "igemm4" --timeout 120 --timeout-method thread \
  > gpurun_out/ig4_tests.log 2>&1 || { tail -40 gpurun_out/ig4_tests.log; exit 1; }
tail -5 gpurun_out/ig4_tests.log
timeout -k 10 400 python -u benchmarks/bench_kernels.py --reps 10 --top 8 ${IG4_BENCH_ARGS} > gpurun_out/ig4_bench.log 2>&1 || { tail -20 gpurun_out/ig4_bench.log; exit 1; }
cat gpurun_out/ig4_bench.log
