#!/bin/bash
# segmented DDP schedules ("concurrent" default vs "serial") with emulated ring collectives
mkdir -p gpurun_out
for cfg in "300 8" "150 8" "300 2"; do
  set -- $cfg
  for s in concurrent serial; do
    echo "busbw=$1 W=$2 $(timeout -k 10 120 python -m benchmarks.phase_timing --schedule $s --fake_busbw_gbs $1 --fake_world $2 2>/dev/null)" || exit 1
  done
done | tee gpurun_out/ddp_sched.txt
