#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py -k narrow -x -q --timeout 120 --timeout-method thread > gpurun_out/narrow2.log 2>&1 || exit 1
timeout -k 10 60 python -m benchmarks.bench_narrow >> gpurun_out/narrow2.log 2>&1 || exit 1
DCGAN_NARROW_VALU=1 timeout -k 10 60 python -m benchmarks.bench_narrow >> gpurun_out/narrow2.log 2>&1 || exit 1
cd gpurun_out
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_VALU SQ_WAIT_ANY -d pmc_n3 -o run -- python -m benchmarks.bench_narrow >> narrow2.log 2>&1 || exit 1
cd ..
for i in 1 2; do
for env in "X=0" "DCGAN_NARROW_VALU=1"; do
echo "[$env]" >> gpurun_out/narrow2.log
env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 >> gpurun_out/narrow2.log 2>&1 || exit 1
done; done
