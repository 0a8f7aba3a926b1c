#!/bin/bash
# round 5, call A: DDP schedule tests + W=1 overhead, then the ping-pong kernels
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_ddp.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/ddp_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/ddp_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
OUT=ddp_ab_r5a.txt bash scripts/gpu_ddp_ab.sh 3 "DCGAN_DDP_GCUT=-1,DCGAN_DDP_GCUT=1" || exit 1
bash scripts/gpu_pp_first.sh
