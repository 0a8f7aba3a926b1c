#!/bin/bash
# GPU tests (kernels + engine), then the bench twice; optional $1 = extra sweep filter for bench_kernels
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -q -m gpu -x --timeout 300 \
  --timeout-method thread > gpurun_out/it3_tests.log 2>&1
rc=$?; tail -4 gpurun_out/it3_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 120 python bench.py --steps 100 --warmup 20 2>/dev/null | cut -c1-330 || exit 1; done
if [ -n "$1" ]; then
  timeout -k 10 600 python -u benchmarks/bench_wgrad.py --batch 128 $1 > gpurun_out/wgrad_it3.log 2>&1 || { tail gpurun_out/wgrad_it3.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/wgrad_it3.log | cut -c1-220
fi
