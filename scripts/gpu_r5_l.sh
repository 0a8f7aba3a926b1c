#!/bin/bash
# round 5: Adam over g_h1's slice right after its collective (DCGAN_ADAM_G_SPLIT) -- DDP GPU tests,
# W=1 force_ddp A/B, RCCL-like stand-in at W=8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_hip_ddp.py \
  > gpurun_out/r5l_ddp_tests.log 2>&1 || { tail -30 gpurun_out/r5l_ddp_tests.log; exit 1; }
tail -2 gpurun_out/r5l_ddp_tests.log
for i in 1 2 3; do for f in 0 1; do
  r=$(DCGAN_ADAM_G_SPLIT=$f timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 --force_ddp 2>/dev/null) || { echo "FAILED $f"; exit 1; }
  echo "force_ddp DCGAN_ADAM_G_SPLIT=$f :: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["schedule"], d["config"]["kernels_per_step"])')"
done; done | tee gpurun_out/ab_adam_g_split_w1.txt
for i in 1 2; do for bw in 150 300; do for w in fp32 bf16; do for f in 0 1; do
  r=$(DCGAN_ADAM_G_SPLIT=$f timeout -k 10 300 python3 -m benchmarks.phase_timing --fake_busbw_gbs $bw --fake_world 8 --allreduce_dtype $w --steps 50 2>/dev/null) || exit 1
  echo "busbw=$bw W=8 wire=$w split=$f $(echo "$r" | tail -1)"
done; done; done; done | tee gpurun_out/ab_adam_g_split_standin.txt
