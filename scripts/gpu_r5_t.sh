#!/bin/bash
# round 5: wgrad5 k-tiles across small images (Wd = 4): tests + 64x64 sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py \
  -k "wgrad5" > gpurun_out/r5t_tests.log 2>&1 || { tail -40 gpurun_out/r5t_tests.log; exit 1; }
tail -2 gpurun_out/r5t_tests.log
timeout -k 10 400 python3 -u benchmarks/bench_wgrad.py --batch 128 --size 64 --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_wgrad5_64e.txt
