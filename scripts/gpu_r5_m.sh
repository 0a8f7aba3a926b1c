#!/bin/bash
# round 5: segmented DDP step -- Adam(G) split (W=1 force_ddp) and the G chain on a high-priority
# stream (DCGAN_G_PRIO), W=1 and the RCCL-like stand-in at W=8
set -o pipefail
mkdir -p gpurun_out
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["schedule"], d["config"]["kernels_per_step"])'; }
for i in 1 2 3; do for v in "DCGAN_ADAM_G_SPLIT=0" "DCGAN_ADAM_G_SPLIT=1" "DCGAN_G_PRIO=1"; do
  r=$(env $v timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 --force_ddp 2>/dev/null) || { echo "FAILED $v"; exit 1; }
  echo "force_ddp $v :: $(echo "$r" | js)"
done; done | tee gpurun_out/ab_ddp_w1_r5m.txt
for i in 1 2; do for w in fp32 bf16; do for f in 0 1; do
  r=$(DCGAN_G_PRIO=$f timeout -k 10 300 python3 -m benchmarks.phase_timing --fake_busbw_gbs 150 --fake_world 8 --allreduce_dtype $w --steps 50 2>/dev/null) || exit 1
  echo "busbw=150 W=8 wire=$w gprio=$f $(echo "$r" | tail -1)"
done; done; done | tee gpurun_out/ab_g_prio_standin.txt
