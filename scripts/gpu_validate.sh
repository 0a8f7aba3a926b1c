#!/bin/bash
# Round validation: full GPU suite, smoke, bench (two lengths), rocprof step profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 180 python bench.py > gpurun_out/bench1.log 2>&1 || exit 1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 >> gpurun_out/bench1.log 2>&1 || exit 1
timeout -k 10 180 python -m benchmarks.phase_timing > gpurun_out/phase_v.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/profV -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/profV.log 2>&1 || exit 1
