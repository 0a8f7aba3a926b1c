#!/bin/bash
# full GPU suite, then interleaved A/B of environment switches on the headline bench ($@ = "VAR:v1 v2" specs)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -6 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for spec in "$@"; do
  bash scripts/gpu_ab_vals.sh "${spec%%:*}" "${spec#*:}" || exit 1
done
exit $rc
