#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py tests/test_functional.py -q -m gpu -x > gpurun_out/k.log 2>&1 || { tail -30 gpurun_out/k.log; exit 1; }
tail -2 gpurun_out/k.log
bash scripts/gpu_stamps.sh
