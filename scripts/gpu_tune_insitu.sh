#!/bin/bash
# in-situ tile tuning by whole-step time under the current schedule (one pass, sibling tiles too)
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m benchmarks.tune_insitu --steps 150 --passes 1 --tiles --out gpurun_out/tuned_insitu.json \
  > gpurun_out/tune_insitu.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/tune_insitu.log | grep -E "keep|incumbent|pass|keys" ; exit $rc
