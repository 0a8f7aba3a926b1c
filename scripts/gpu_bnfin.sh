#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -x -q --timeout 120 --timeout-method thread \
  -k "bn or stagewise or step_matches or graph_replay" > gpurun_out/bnfin_tests.log 2>&1 || { tail -30 gpurun_out/bnfin_tests.log; exit 1; }
tail -2 gpurun_out/bnfin_tests.log
bash scripts/gpu_ab_env.sh DCGAN_OLD_BNFIN "0 1" 3
