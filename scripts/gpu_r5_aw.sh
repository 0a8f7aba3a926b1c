#!/bin/bash
# round 5: DDP step with D's gradient in three collectives (DCGAN_DDP_DMID): RCCL tests, W=1 A/B, stand-in W=2/4/8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_hip_ddp.py -m gpu -x -q --timeout 240 --timeout-method thread -k "rccl_single_rank" > gpurun_out/gpu_tests_ddp_dmid_r5.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_ddp_dmid_r5.log; [ $rc -eq 0 ] || exit $rc
ab=gpurun_out/ab_ddp_dmid_r5.txt; : > $ab
for r in 1 2; do
  for w in 8 4 2; do
    for v in 0 1; do
      for wire in fp32 bf16; do
        x=$(DCGAN_DDP_DMID=$v timeout -k 10 150 python3 -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --fake_world $w --allreduce_dtype $wire 2>/dev/null | grep '^{') || exit 1
        echo "standin W=$w $wire dmid=$v $x" >> $ab
      done
    done
  done
done
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for r in 1 2; do
  for v in 0 1; do
    x=$(DCGAN_DDP_DMID=$v timeout -k 10 150 python3 bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "W=1 force_ddp dmid=$v :: $x" >> $ab
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_ddp_dmid_r5.txt'):
    if 'standin' in l:
        pre, js = l.split('{', 1); d = json.loads('{' + js); print(pre.strip(), d['ms_per_step_timed'])
    else:
        print(l.rstrip())
PY
