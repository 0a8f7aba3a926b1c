#!/bin/bash
# quick check after a kernel change: selected GPU tests ($1 = -k expr), then bench twice
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread ${1:+-k "$1"} \
  > gpurun_out/gpu_quick.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_quick.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 180 python bench.py --steps 200 --warmup 20 2>/dev/null | cut -c1-260 || exit 1; done
