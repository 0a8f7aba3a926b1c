#!/bin/bash
# quick: selected GPU tests (-k), then bench + kernel-trace profile
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x ${1:+-k "$1"} > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python bench.py --steps 20 --warmup 3 > gpurun_out/prof3.log 2>&1 || { tail -20 gpurun_out/prof3.log; exit 1; }
