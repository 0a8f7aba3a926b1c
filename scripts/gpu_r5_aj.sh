#!/bin/bash
# round 5: segmented DDP step with G weight gradients on alt1 (DCGAN_DDP_GW_ALT, G slice above g_h1 reduced from alt1) -- RCCL
# bit-identity tests, W=1 force_ddp A/B (eager), RCCL-like stand-in at W=8 (eager)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_hip_ddp.py -m gpu -x -q --timeout 240 --timeout-method thread -k "rccl_single_rank" > gpurun_out/gpu_tests_ddp_gw_alt_b_r5.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_ddp_gw_alt_b_r5.log; [ $rc -eq 0 ] || exit $rc
ab=gpurun_out/ab_ddp_gw_alt_b_r5.txt; : > $ab
for r in 1 2; do
  for v in 0 1 2; do
    x=$(DCGAN_DDP_GW_ALT=$v timeout -k 10 150 python3 bench.py --force_ddp --steps 100 --warmup 20 2>/dev/null | grep '^{' | cut -c1-400) || exit $?
    echo "round $r force_ddp W=1 gw_alt=$v $x" >> $ab
  done
done
for r in 1 2; do
  for v in 0 1 2; do
    for w in fp32 bf16; do
      x=$(DCGAN_DDP_GW_ALT=$v timeout -k 10 150 python3 -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --allreduce_dtype $w 2>/dev/null | grep '^{') || exit $?
      echo "round $r standin W=8 busbw=150 wire=$w gw_alt=$v $x" >> $ab
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_ddp_gw_alt_b_r5.txt'):
    pre, js = l.split('{', 1); d = json.loads('{' + js) if js.rstrip().endswith('}') else {}
    print(pre.strip(), d.get('value') and round(d['value']), d.get('ms_per_step') or d.get('ms_per_step_timed'))
PY
