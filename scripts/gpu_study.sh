#!/bin/bash
# igemm4 ablation study ($@ passed to benchmarks/ig4_study.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/ig4_study.py "$@" > gpurun_out/ig4_study.log 2>&1 || { tail -20 gpurun_out/ig4_study.log; exit 1; }
cat gpurun_out/ig4_study.log
