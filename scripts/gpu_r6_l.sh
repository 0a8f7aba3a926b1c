#!/bin/bash
# round 6: Adam(D) on the D chain's stream beside the G tail in the all-reduce DDP step
# (DCGAN_DDP_ADAM_D_ALT) -- DDP GPU tests, RCCL-like stand-in A/B at W = 8 / 4 / 2, --force_ddp vs fused
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_ddp.py -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r6l.log 2>&1
rc=$?; echo "ddp tests rc=$rc"; tail -3 gpurun_out/gpu_tests_r6l.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c 'import json,sys
for l in sys.stdin:
    l=l.strip()
    if l.startswith("{"):
        d=json.loads(l); print(d.get("value"), d.get("ms_per_step"), d.get("ms_per_step_timed",""), json.dumps(d.get("phases_ms","")))'; }
for i in 1 2; do
  for W in 8 4 2; do
    for a in 1 0; do
      r=$(DCGAN_DDP_ADAM_D_ALT=$a timeout -k 10 120 python -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --fake_world $W --steps 50 --warmup 20 2>/dev/null) || exit 1
      echo "standin W=$W busbw=150 wire=fp32 adam_d_alt=$a $(echo "$r" | val)"
    done
  done
done | tee gpurun_out/ab_ddp_adam_d_alt_standin_r6.txt
for i in 1 2 3; do
  for a in 1 0; do
    r=$(DCGAN_DDP_ADAM_D_ALT=$a timeout -k 10 120 python bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null) || exit 1; echo "[force_ddp adam_d_alt=$a] $(echo "$r" | val)"
  done
  r=$(timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null) || exit 1; echo "[fused] $(echo "$r" | val)"
done | tee gpurun_out/ab_ddp_adam_d_alt_w1_r6.txt
