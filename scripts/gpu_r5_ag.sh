#!/bin/bash
# round 5: placement tests on the GPU; G weight gradients beside the chains at 128x128 / 256x256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_hip_engine.py tests/test_hip_ddp.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_place_r5.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_place_r5.log; [ $rc -eq 0 ] || exit $rc
ab=gpurun_out/ab_gw_place_128_256_r5.txt; : > $ab
for r in 1 2; do
  for v in 0 1; do
    x=$(DCGAN_G_WGRAD_ON_D=$v timeout -k 10 200 python3 bench.py --output_size 128 --steps 40 --warmup 10 2>/dev/null | grep '^{') || exit $?
    echo "round $r 128 bf16 g_wgrad_beside=$v $x" >> $ab
    x=$(DCGAN_G_WGRAD_ON_D=$v timeout -k 10 200 python3 bench.py --output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3 2>/dev/null | grep '^{') || exit $?
    echo "round $r 256 fp16 g_wgrad_beside=$v $x" >> $ab
  done
done
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | grep '^{' | cut -c75-140; done | tee gpurun_out/bench_driver_form_place_r5.txt
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_gw_place_128_256_r5.txt'):
    pre, js = l.split('{', 1); d = json.loads('{' + js)
    print(pre.strip(), round(d['value']), d['ms_per_step'])
PY
