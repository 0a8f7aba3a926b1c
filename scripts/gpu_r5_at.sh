#!/bin/bash
# round 5: DDP g_h1 weight-gradient placement (1 = cs, 2 = alt1) under the stand-in at W=2 and W=4 (150 GB/s), fp32 wire
set -o pipefail
mkdir -p gpurun_out
ab=gpurun_out/ab_ddp_gw_world_r5.txt; : > $ab
for r in 1 2; do
  for w in 2 4 8; do
    for v in 1 2; do
      x=$(DCGAN_DDP_GW_ALT=$v timeout -k 10 150 python3 -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --fake_world $w 2>/dev/null | grep '^{') || exit 1
      echo "standin W=$w busbw=150 wire=fp32 gw_alt=$v $x" >> $ab
    done
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_ddp_gw_world_r5.txt'):
    pre, js = l.split('{', 1); d = json.loads('{' + js)
    print(pre.strip(), d['ms_per_step_timed'])
PY
