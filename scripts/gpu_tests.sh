#!/bin/bash
# Full GPU test suite only (stop at the first fault / timeout).
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -q -m gpu -x ${1:+-k "$1"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -25 gpurun_out/gpu_tests.log
exit $rc
