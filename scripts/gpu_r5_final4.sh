#!/bin/bash
# round 5 final (4): smoke(), full GPU suite, headline bench (200/20 and the driver's 20/5 form)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5_final4.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_r5_final4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r5_final4.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r5_final4.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | grep '^{' | cut -c75-160; done | tee gpurun_out/bench_r5_final4.txt
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | grep '^{' | cut -c75-160; done | tee -a gpurun_out/bench_r5_final4.txt
