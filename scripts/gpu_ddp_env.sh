#!/bin/bash
# One-graph DDP with emulated collectives under HIP queue settings.
mkdir -p gpurun_out
run() { timeout -k 10 120 "$@" 2>/dev/null || exit 1; }
for e in "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8 DEBUG_HIP_FORCE_GRAPH_QUEUES=8" "GPU_MAX_HW_QUEUES=16 DEBUG_HIP_FORCE_GRAPH_QUEUES=16"; do
  echo "== $e"
  run env $e python -m benchmarks.phase_timing --schedule ddp --fake_busbw_gbs 300
  run env $e python -m benchmarks.phase_timing --schedule concurrent --fake_busbw_gbs 300
  run env $e python bench.py --steps 200 --warmup 20 | cut -c1-200
done 2>&1 | tee gpurun_out/ddp_env2.txt
