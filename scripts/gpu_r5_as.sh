#!/bin/bash
# round 5: DDP g_h1 weight-gradient placement (DCGAN_DDP_GW_ALT 1 = cs, 3 = side stream): RCCL tests, W=1 A/B, W=8 stand-in
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_hip_ddp.py -m gpu -x -q --timeout 240 --timeout-method thread -k "rccl_single_rank" > gpurun_out/gpu_tests_ddp_mode3_r5.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_ddp_mode3_r5.log; [ $rc -eq 0 ] || exit $rc
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
ab=gpurun_out/ab_ddp_gw_mode3_r5.txt; : > $ab
for r in 1 2 3; do
  for v in 1 3; do
    x=$(DCGAN_DDP_GW_ALT=$v timeout -k 10 150 python3 bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null | js) || exit 1
    echo "W=1 force_ddp gw_alt=$v :: $x" >> $ab
  done
done
for r in 1 2; do
  for v in 1 3; do
    for w in fp32 bf16; do
      x=$(DCGAN_DDP_GW_ALT=$v timeout -k 10 150 python3 -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --allreduce_dtype $w 2>/dev/null | grep '^{') || exit 1
      echo "standin W=8 busbw=150 wire=$w gw_alt=$v $x" >> $ab
    done
  done
done
cut -c1-150 $ab
