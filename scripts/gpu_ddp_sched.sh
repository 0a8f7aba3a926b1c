#!/bin/bash
# DDP-schedule checks on one GPU: the 2-rank DDP tests (gloo) + the concurrent schedule's timeline
# with emulated collectives (G 150 us, D top 60 us, D rest 20 us)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread -k "ddp or engine" \
  > gpurun_out/gpu_quick.log 2>&1 || { tail -20 gpurun_out/gpu_quick.log; exit 1; }
tail -1 gpurun_out/gpu_quick.log
timeout -k 10 200 python -m benchmarks.phase_timing 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -m benchmarks.phase_timing --fake_comm_us 150,60,20 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -m benchmarks.phase_timing --fake_comm_us 300,120,40 2>&1 | grep -v amdgpu.ids || exit 1
