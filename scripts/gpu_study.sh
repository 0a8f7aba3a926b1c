#!/bin/bash
# igemm4 vs igemm3 per layer (production build: ablation 0 only). Args: "layer refs" pairs.
mkdir -p gpurun_out
CF=500,501,502,503,504,505,506,507,510,511,512,513,514,515,516,517
for spec in "$@"; do
  set -- $spec
  timeout -k 10 120 python -u benchmarks/ig4_study.py --only $1 --cfgs $CF --ablate 0 --ref $2 \
    >> gpurun_out/ig4_study.log 2>&1 || { tail -20 gpurun_out/ig4_study.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ig4_study.log
