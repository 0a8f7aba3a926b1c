#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py -k narrow -x -q --timeout 120 --timeout-method thread > gpurun_out/narrow3.log 2>&1 || exit 1
DCGAN_NARROW_WLDS=1 timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py -k narrow -x -q --timeout 120 --timeout-method thread >> gpurun_out/narrow3.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 60 python -m benchmarks.bench_narrow >> gpurun_out/narrow3.log 2>&1 || exit 1
DCGAN_NARROW_WLDS=1 timeout -k 10 60 python -m benchmarks.bench_narrow >> gpurun_out/narrow3.log 2>&1 || exit 1
done
