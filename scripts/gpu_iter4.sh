#!/bin/bash
# GPU tests (kernels + engine), then bench x2 + kernel-trace profile ($1 = tag)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -q -m gpu -x --timeout 300 \
  --timeout-method thread > gpurun_out/it4_tests.log 2>&1
rc=$?; tail -4 gpurun_out/it4_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_prof_step.sh ${1:-cur}
