#!/bin/bash
# round 5: wgrad5 Wd=64 tile test; per-layer weight-gradient sweeps at 128x128 and 256x256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py \
  -k "wgrad5" > gpurun_out/r5r_tests.log 2>&1 || { tail -40 gpurun_out/r5r_tests.log; exit 1; }
tail -2 gpurun_out/r5r_tests.log
timeout -k 10 500 python3 -u benchmarks/bench_wgrad.py --batch 128 --size 128 --reps 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_wgrad5_128.txt
timeout -k 10 600 python3 -u benchmarks/bench_wgrad.py --batch 512 --size 256 --reps 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_wgrad5_256.txt
