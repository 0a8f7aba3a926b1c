#!/bin/bash
# in-situ tile tuning by whole-step time: $1 = output tag, remaining args -> benchmarks.tune_insitu
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 1100 python -u -m benchmarks.tune_insitu --out gpurun_out/tuned_$tag.json "$@" \
  > gpurun_out/tune_$tag.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/tune_$tag.log | grep -E "keep|incumbent|pass|keys|seed|failed" ; exit $rc
