#!/bin/bash
# round 6 (a): driver-form anatomy (per-step events) + the driver's exact command x3
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 240 python3 -u benchmarks/study/driver_per_step.py --steps 20 --warmup 5 --repeat 3 > gpurun_out/r6/driver_per_step.txt 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | grep '^{' | cut -c75-140; done | tee gpurun_out/r6/bench_driver_form_a.txt
