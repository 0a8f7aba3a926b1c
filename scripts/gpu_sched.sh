#!/bin/bash
# DDP schedules on one GPU with emulated collective latencies (G, D-top, D-rest all-reduce).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/phase.log
for fc in "" "150,100,30" "300,200,60"; do
for env in "X=0" "DCGAN_DDP_SCHEDULE=hybrid" "DCGAN_SERIAL_DBWD=1"; do
env $env timeout -k 10 120 python -m benchmarks.phase_timing ${fc:+--fake_comm_us $fc} >> gpurun_out/phase.log 2>&1 || exit 1
done; done
