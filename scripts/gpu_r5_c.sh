#!/bin/bash
# round 5, call C: eager vs graph for the fused and the DDP schedules (W=1), copy-free vs copying bf16 wire
mkdir -p gpurun_out
out=gpurun_out/sched_eager_r5c.txt; : > $out
val() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"], d["config"]["graphs_per_step"], d["config"]["schedule"])'; }
for i in 1 2; do
  for spec in "--graph 1" "--graph 0" "--force_ddp --graph 1" "--force_ddp --graph 0" \
              "DCGAN_DDP_SCHEDULE=ddp --force_ddp --graph 1" "DCGAN_DDP_SCHEDULE=ddp --force_ddp --graph 0" \
              "--force_ddp --allreduce_dtype bf16" "DCGAN_WIRE_DIRECT=0 --force_ddp --allreduce_dtype bf16"; do
    envs=$(echo "$spec" | tr ' ' '\n' | grep '=' | grep -v '^--' | tr '\n' ' ')
    args=$(echo "$spec" | tr ' ' '\n' | grep -v '^DCGAN' | tr '\n' ' ')
    r=$(env $envs timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 $args 2>/dev/null) || { echo "failed: $spec" | tee -a $out; exit 1; }
    echo "$spec :: $(echo "$r" | val)" | tee -a $out
  done
done
