#!/bin/bash
# Full GPU test suite (one process), then an A/B (arg 1: env toggle) and a step profile.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
bash scripts/gpu_abprof.sh "${1:-X=1}" ${2:-profF}
