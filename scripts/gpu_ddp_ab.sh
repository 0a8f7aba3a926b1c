#!/bin/bash
# DDP step vs fused step on one box: $1 interleaved pairs of bench.py (fused) / bench.py --force_ddp
# (one-rank RCCL group, segmented schedule), then optional env variants of the DDP step ($2: "A=1 B=2,...").
mkdir -p gpurun_out
out=gpurun_out/${OUT:-ddp_ab.txt}
: > $out
val() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"], d["config"]["graphs_per_step"])'; }
for i in $(seq 1 ${1:-3}); do
  r=$(timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 2>/dev/null) || { echo "fused failed" >> $out; exit 1; }
  echo "fused :: $(echo "$r" | val)" | tee -a $out
  r=$(timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 --force_ddp 2>/dev/null) || { echo "ddp failed" >> $out; exit 1; }
  echo "ddp :: $(echo "$r" | val)" | tee -a $out
  IFS=',' read -ra VARS <<< "${2:-}"
  for v in "${VARS[@]}"; do
    r=$(env $v timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 --force_ddp 2>/dev/null) || { echo "ddp $v failed" >> $out; exit 1; }
    echo "ddp $v :: $(echo "$r" | val)" | tee -a $out
  done
done
