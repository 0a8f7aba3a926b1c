#!/bin/bash
# round 6: all-reduce DDP step -- Adam over g_h2..g_h4 with g_h1's slice (DCGAN_ADAM_G_EARLY_B),
# Adam(D) on the D stream (DCGAN_DDP_ADAM_D_ALT); DDP GPU tests first
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hip_ddp.py -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r6m.log 2>&1
rc=$?; echo "ddp tests rc=$rc"; tail -3 gpurun_out/gpu_tests_r6m.log; [ $rc -eq 0 ] || exit $rc
./scripts/gpu_standin_ab.sh DCGAN_ADAM_G_EARLY_B "1 0" || exit 1
DCGAN_ADAM_G_EARLY_B=1 ./scripts/gpu_standin_ab.sh DCGAN_DDP_ADAM_D_ALT "1 0"
