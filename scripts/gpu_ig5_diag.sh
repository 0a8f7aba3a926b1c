#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u benchmarks/study/ig5_diag.py 4 16 128 256 400,401,402,403,411,412,413 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ig5_diag.log
