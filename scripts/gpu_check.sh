#!/bin/bash
# Targeted GPU tests ($1 = pytest -k expr or test files) then the config benches.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $1 -x -v --timeout 300 --timeout-method thread > gpurun_out/check_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/check_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
for d in 1 0; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --defer_update $d 2>/dev/null | cut -c1-300 || exit 1
done
bash scripts/gpu_configs.sh
