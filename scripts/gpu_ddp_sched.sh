#!/bin/bash
# DDP schedules ("concurrent" default, "serial", one-graph "ddp") with the RCCL-like stand-in
# (csrc/hip/comm_emu.hip: 32 workgroups moving 2(W-1)/W x bytes through HBM, paced to the ring
# model) at each collective's call point; plus the fused single-GPU step for reference.
# A failing step ends the script.
mkdir -p gpurun_out
out=gpurun_out/ddp_sched.txt
: > $out
run() {  # label, phase_timing args
  local label=$1; shift
  local r
  r=$(timeout -k 10 120 python -m benchmarks.phase_timing "$@" 2>gpurun_out/ddp_sched.err) || { echo "FAILED: $label"; tail -5 gpurun_out/ddp_sched.err; exit 1; }
  echo "$label $r" | tee -a $out
}
run fused
for cfg in "300 8 fp32" "150 8 fp32" "150 8 bf16" "300 2 fp32"; do
  set -- $cfg
  for s in concurrent serial ddp; do
    run "busbw=$1 W=$2 wire=$3" --schedule $s --fake_busbw_gbs $1 --fake_world $2 --allreduce_dtype $3 ${FAKE_ARGS}
  done
done
