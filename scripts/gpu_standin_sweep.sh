#!/bin/bash
# DDP step under the RCCL-like stand-in: bus bandwidth x wire sweep at W = 8 / 4 / 2 (current defaults)
mkdir -p gpurun_out
val() { python3 -c 'import json,sys
for l in sys.stdin:
    l=l.strip()
    if l.startswith("{"):
        d=json.loads(l); print(d.get("ms_per_step_timed",""), json.dumps(d.get("phases_ms","")))'; }
for W in 8 4 2; do for bw in 150 300; do for wire in fp32 bf16; do
  r=$(timeout -k 10 120 python -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs $bw --fake_world $W --allreduce_dtype $wire --steps 50 --warmup 20 2>/dev/null) || exit 1
  echo "standin W=$W busbw=$bw wire=$wire $(echo "$r" | val)"
done; done; done | tee gpurun_out/standin_sweep.txt
