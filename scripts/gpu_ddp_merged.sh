#!/bin/bash
# DDP step: Adam(D) merged into the final adam2 (DCGAN_DDP_ADAM_D_ALT=m) vs on the D stream (1):
# bit-exactness test, then the stand-in / --force_ddp A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_ddp.py -q -x -k "merged or two_ranks_match" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_merged.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_merged.log; [ $rc -eq 0 ] || exit $rc
./scripts/gpu_standin_ab.sh DCGAN_DDP_ADAM_D_ALT "1 m"
