#!/bin/bash
# A/B of one HipEngine switch (see the echo lines): 1 vs 0, alternating
mkdir -p gpurun_out
FLAG=${1:?usage: gpu_ab_switch.sh HipEngine_switch}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "${2:-engine or ddp or trainer or linear}" \
  > gpurun_out/gpu_quick.log 2>&1 || { tail -20 gpurun_out/gpu_quick.log; exit 1; }
tail -1 gpurun_out/gpu_quick.log
for i in 1 2; do
  for v in 1 0; do
    echo -n "$FLAG=$v "
    timeout -k 10 180 python -m benchmarks.ab_engine_flag $FLAG $v --steps 200 --warmup 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['config']['kernels_per_step'])" || exit 1
  done
done
