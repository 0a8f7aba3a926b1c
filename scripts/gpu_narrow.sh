#!/bin/bash
# MFMA narrow deconv: kernel tests (MFMA and, via env, the VALU kernel), A/B bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py -k narrow -x -v --timeout 120 --timeout-method thread > gpurun_out/narrow_tests.log 2>&1 || exit 1
DCGAN_NARROW_VALU=1 timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py -k narrow -x -q --timeout 120 --timeout-method thread >> gpurun_out/narrow_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_hip_engine.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/narrow_tests.log 2>&1 || exit 1
: > gpurun_out/narrow_ab.log
for i in 1 2 3; do
for env in "X=0" "DCGAN_NARROW_VALU=1"; do
echo "[$env]" >> gpurun_out/narrow_ab.log
env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 >> gpurun_out/narrow_ab.log 2>&1 || exit 1
done; done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_narrow -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/prof_narrow.log 2>&1 || exit 1
