#!/bin/bash
# Step anatomy: (1) per-phase timeline of the concurrent schedule, (2) kernel trace of the
# serial schedule (every kernel alone on the GPU: isolated durations inside the real step).
mkdir -p gpurun_out
timeout -k 10 180 python -m benchmarks.phase_timing > gpurun_out/phase.log 2>&1 || { tail -20 gpurun_out/phase.log; exit 1; }
tail -2 gpurun_out/phase.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_serial
DCGAN_SERIAL_DBWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/prof_serial.log 2>&1 || { tail -20 gpurun_out/prof_serial.log; exit 1; }
tail -1 gpurun_out/prof_serial.log
