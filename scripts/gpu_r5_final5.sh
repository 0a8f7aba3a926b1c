#!/bin/bash
# round 5 final (5): full GPU suite, then every config's bench line + driver form + one-rank DDP
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r5_final5.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r5_final5.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/bench_configs_r5_final5.jsonl
for args in "--steps 200 --warmup 20" "--dtype fp16 --steps 50 --warmup 10" "--dtype fp32 --steps 20 --warmup 5" \
            "--output_size 28 --c_dim 1 --steps 30 --warmup 5" "--output_size 128 --steps 20 --warmup 5" \
            "--output_size 256 --batch_size 512 --dtype fp16 --steps 10 --warmup 3"; do
  timeout -k 10 300 python3 bench.py $args 2>/dev/null | grep '^{' >> gpurun_out/bench_configs_r5_final5.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/bench_configs_r5_final5.jsonl'):
    d=json.loads(l); print(d['config']['model'][:22], d['dtype'], d['value'], d['ms_per_step'])"
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | grep '^{' | cut -c75-140; done | tee gpurun_out/bench_driver_form_r5_final5.txt
for i in 1 2; do timeout -k 10 120 python3 bench.py --force_ddp --steps 50 --warmup 10 2>/dev/null | grep '^{' | cut -c75-140; done | tee gpurun_out/bench_force_ddp_r5_final5.txt
