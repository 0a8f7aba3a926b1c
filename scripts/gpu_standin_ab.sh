#!/bin/bash
# A/B of an environment variable on the DDP step under the RCCL-like stand-in
# (benchmarks/phase_timing.py: fp32 wire, 150 GB/s, eager) at W = 8 / 4 / 2, interleaved x2, then
# bench.py --force_ddp (one-rank RCCL group) per value vs the fused step, interleaved x3.
# $1 = VAR, $2 = "v1 v2 ..."; output gpurun_out/standin_<VAR>.txt
mkdir -p gpurun_out
var=$1; vals=$2
val() { python3 -c 'import json,sys
for l in sys.stdin:
    l=l.strip()
    if l.startswith("{"):
        d=json.loads(l); print(d.get("value"), d.get("ms_per_step"), d.get("ms_per_step_timed",""), json.dumps(d.get("phases_ms","")))'; }
{ for i in 1 2; do for W in 8 4 2; do for v in $vals; do
    r=$(env $var=$v timeout -k 10 120 python -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --fake_world $W --steps 50 --warmup 20 2>/dev/null) || exit 1
    echo "standin W=$W $var=$v $(echo "$r" | val)"
  done; done; done
  for i in 1 2 3; do
    for v in $vals; do
      r=$(env $var=$v timeout -k 10 120 python bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null) || exit 1; echo "[force_ddp $var=$v] $(echo "$r" | val)"
    done
    r=$(timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null) || exit 1; echo "[fused] $(echo "$r" | val)"
  done; } | tee gpurun_out/standin_$var.txt
