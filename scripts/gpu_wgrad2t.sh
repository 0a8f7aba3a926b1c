#!/bin/bash
# wgrad3 two-tap tiles: numerics, then the per-layer wgrad sweep (bench_wgrad, incl. 320..333)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "wgrad3" > gpurun_out/w2t_tests.log 2>&1 || { tail -30 gpurun_out/w2t_tests.log; exit 1; }
tail -2 gpurun_out/w2t_tests.log
timeout -k 10 400 python -u benchmarks/bench_wgrad.py --batch 128 --reps 10 > gpurun_out/w2t_sweep.log 2>&1 || { tail -20 gpurun_out/w2t_sweep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/w2t_sweep.log | cut -c1-250
