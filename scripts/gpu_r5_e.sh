#!/bin/bash
# round 5, call E: driver-form A/B eager vs graph (5 pairs), then the whole GPU suite
mkdir -p gpurun_out
out=gpurun_out/eager_graph_driverform_r5e.txt; : > $out
val() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"], d["config"]["hip_graph"])'; }
for i in 1 2 3 4 5; do
  for g in 0 1; do
    r=$(timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --graph $g 2>/dev/null) || { echo "bench failed" >> $out; exit 1; }
    echo "graph=$g :: $(echo "$r" | val)" | tee -a $out
  done
done
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5e.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_r5e.log; exit $rc
