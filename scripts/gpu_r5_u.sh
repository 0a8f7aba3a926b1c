#!/bin/bash
# round 5 checkpoint: full GPU suite, driver-form bench, step kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r5u.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r5u.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | grep '^{' | cut -c1-140; done | tee gpurun_out/bench_driver_form_r5u.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r5u
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5u -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_r5u.log 2>&1 || { tail -5 gpurun_out/prof_r5u.log; exit 1; }
echo profiled
