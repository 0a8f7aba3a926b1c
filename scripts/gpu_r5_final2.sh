#!/bin/bash
# round 5 final (2): full GPU suite, then every config's bench line + driver form + one-rank DDP
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r5_final.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r5_final.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r5_final.sh
