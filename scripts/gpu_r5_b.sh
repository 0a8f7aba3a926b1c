#!/bin/bash
# round 5, call B: DDP tests (7-segment schedule + copy-free bf16 wire), W=1 overhead, stand-in at W=8
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_ddp.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/ddp_tests_b.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/ddp_tests_b.log | tail -20; [ $rc -eq 0 ] || exit $rc
OUT=ddp_ab_r5b.txt bash scripts/gpu_ddp_ab.sh 2 "" || exit 1
: > gpurun_out/standin_r5b.txt
for w in fp32 bf16; do
  r=$(timeout -k 10 300 python3 -m benchmarks.phase_timing --fake_busbw_gbs 150 --fake_world 8 --allreduce_dtype $w --steps 50 2>/dev/null) || exit 1
  echo "busbw=150 W=8 wire=$w $r" | tee -a gpurun_out/standin_r5b.txt
done
