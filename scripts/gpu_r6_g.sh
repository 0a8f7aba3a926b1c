#!/bin/bash
# round 6: sharded DDP update -- DDP GPU tests, RCCL-like stand-in (eager, fp32 wire, 150 GB/s) at
# W = 2 / 4 / 8 sharded vs all-reduce, interleaved; --force_ddp (one-rank RCCL) vs fused
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_ddp.py -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r6g.log 2>&1
rc=$?; echo "ddp tests rc=$rc"; tail -3 gpurun_out/gpu_tests_r6g.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for W in 8 4 2; do
    for sh in 1 0; do
      r=$(DCGAN_DDP_SHARD=$sh timeout -k 10 120 python -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --fake_world $W --steps 50 --warmup 20 2>/dev/null) || exit 1
      echo "standin W=$W busbw=150 wire=fp32 shard=$sh $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step_timed"], json.dumps(d["phases_ms"]))')"
    done
  done
done | tee gpurun_out/ab_ddp_shard_standin_r6.txt
for i in 1 2 3; do
  for sh in 1 0; do
    r=$(DCGAN_DDP_SHARD=$sh timeout -k 10 120 python bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null) || exit 1; echo "[force_ddp shard=$sh] ${r:70:40}"
  done
  r=$(timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null) || exit 1; echo "[fused] ${r:70:40}"
done | tee gpurun_out/ab_ddp_shard_w1_r6.txt
./scripts/gpu_ab_vals.sh DCGAN_GW_PLACE "aaaa aaac aaas"
