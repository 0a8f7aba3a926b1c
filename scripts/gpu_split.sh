#!/bin/bash
# Split D forward (D(real) beside G's forward): engine tests, A/B bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_hip_engine.py tests/test_hip_ddp.py tests/test_hip_trainer.py -x -v --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || exit 1
: > gpurun_out/split_ab.log
for i in 1 2 3; do
for env in "X=0" "DCGAN_SPLIT_DFWD=1"; do
echo "[$env]" >> gpurun_out/split_ab.log
env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 >> gpurun_out/split_ab.log 2>&1 || exit 1
done; done
timeout -k 10 120 python -m benchmarks.phase_timing >> gpurun_out/split_ab.log 2>&1 || exit 1
