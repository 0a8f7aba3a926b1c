#!/bin/bash
# narrow2.hip: numerics (nconv / nwgrad vs the fp32 oracle) then timings vs the round-1 paths.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "nconv or nwgrad or conv3 or narrow" > gpurun_out/narrow2_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/narrow2_tests.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -m benchmarks.bench_narrow2 > gpurun_out/narrow2_bench.log 2>&1 || { tail -20 gpurun_out/narrow2_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/narrow2_bench.log
