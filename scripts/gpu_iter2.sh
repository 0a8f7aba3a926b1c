#!/bin/bash
# kernel + engine GPU tests, per-GEMM sweep of the tuned tiles, bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -q -m gpu -x --timeout 300 \
  --timeout-method thread > gpurun_out/it2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/it2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u benchmarks/bench_kernels.py --batch 128 --reps 10 --top 6 --v1 --cfgs 1,2 \
  --out gpurun_out/tuned_it2.json > gpurun_out/tune_it2.log 2>&1 || { tail gpurun_out/tune_it2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tune_it2.log | cut -c1-220
for i in 1 2; do timeout -k 10 120 python bench.py --steps 100 --warmup 20 2>/dev/null | cut -c1-200 || exit 1; done
