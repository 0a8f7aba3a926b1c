#!/bin/bash
# round 5, call F: fused-Adam numerics, Adam / engine tests, then A/B fused-Adam on vs off (driver form + 50/10)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_engine.py tests/test_hip_kernels.py -x -v --timeout 300 --timeout-method thread \
  -k "adam or wgrad or engine" > gpurun_out/tests_f.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" gpurun_out/tests_f.log | tail -20; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/ab_wgrad_adam_r5f.txt; : > $out
val() { python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"], d["config"]["kernels_per_step"])'; }
for i in 1 2 3 4; do
  for a in 1 0; do
    for st in "--steps 20 --warmup 5" "--steps 50 --warmup 10"; do
      r=$(DCGAN_WGRAD_ADAM=$a timeout -k 10 180 python3 bench.py $st 2>/dev/null) || { echo "bench failed" >> $out; exit 1; }
      echo "WGRAD_ADAM=$a $st :: $(echo "$r" | val)" | tee -a $out
    done
  done
done
