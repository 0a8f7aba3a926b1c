#!/bin/bash
# round 5: first Adam part on the G weight gradients' stream (DCGAN_ADAM_SPLIT_ALT): placement
# tests, interleaved 64x64 / 128x128 A/B, tail timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_hip_engine.py -m gpu -x -q --timeout 240 --timeout-method thread -k "placements or early_adam" > gpurun_out/gpu_tests_adam_alt_r5.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_adam_alt_r5.log; [ $rc -eq 0 ] || exit $rc
ab=gpurun_out/ab_adam_split_alt_r5.txt; : > $ab
for r in 1 2 3; do
  for v in 1 0; do
    x=$(DCGAN_ADAM_SPLIT_ALT=$v timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | grep '^{') || exit $?
    echo "round $r 64 adam_split_alt=$v $x" >> $ab
  done
done
for r in 1 2; do
  for v in 1 0; do
    x=$(DCGAN_ADAM_SPLIT_ALT=$v timeout -k 10 200 python3 bench.py --output_size 128 --steps 40 --warmup 10 2>/dev/null | grep '^{') || exit $?
    echo "round $r 128 adam_split_alt=$v $x" >> $ab
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_adam_split_alt_r5.txt'):
    pre, js = l.split('{', 1); d = json.loads('{' + js)
    print(pre.strip(), round(d['value']), d['ms_per_step'])
PY
