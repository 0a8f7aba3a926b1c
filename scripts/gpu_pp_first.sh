#!/bin/bash
# ping-pong K loop: numerics first (stop on any failure), then isolated per-layer timings
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "pipeline_tails or pingpong" > gpurun_out/pp_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Error" gpurun_out/pp_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u benchmarks/bench_kernels.py --batch 128 --size 64 --reps 10 --cfgs 21,24,25,20 --top 8 \
  > gpurun_out/pp_bench64.txt 2>&1 || { tail -5 gpurun_out/pp_bench64.txt; exit 1; }
cat gpurun_out/pp_bench64.txt
