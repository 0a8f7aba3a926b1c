#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -x -q --timeout 120 --timeout-method thread \
  -k "head or nconv or stagewise or step_matches" > gpurun_out/r2b_tests.log 2>&1 || { tail -30 gpurun_out/r2b_tests.log; exit 1; }
tail -1 gpurun_out/r2b_tests.log
bash scripts/gpu_ab_env.sh DCGAN_HEAD_RS "4 1 2" 2 || exit 1
bash scripts/gpu_ab_env.sh DCGAN_NCONV_GRID_G "0 512" 2 || exit 1
bash scripts/gpu_ab_env.sh DCGAN_NWGRAD_CPW_G "1 2 4" 2 || exit 1
bash scripts/gpu_ab_env.sh DCGAN_NWGRAD_CPW_D "1 2 4" 2
