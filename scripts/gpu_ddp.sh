#!/bin/bash
# DDP validation on one GPU: the DDP tests (gloo W=2, one-rank RCCL incl. the one-graph schedule),
# bench with a forced one-rank RCCL group, and the DDP schedules with emulated ring collectives.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_ddp.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/ddp_tests.log 2>&1
rc=$?; tail -15 gpurun_out/ddp_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null | cut -c1-420 || exit 1
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --force_ddp 2>/dev/null | cut -c1-420 || exit 1
done
for bw in 0 300 150; do
  for s in ddp concurrent; do
    timeout -k 10 120 python -m benchmarks.phase_timing --schedule $s --fake_busbw_gbs $bw 2>/dev/null || exit 1
  done
done | tee gpurun_out/ddp_fake_comm.jsonl
