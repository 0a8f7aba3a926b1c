#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -q -m gpu -x -k igemm3 > gpurun_out/k.log 2>&1 || { tail -30 gpurun_out/k.log; exit 1; }
tail -1 gpurun_out/k.log
for sc in "D1.fwd 210:1,215:1" "D3.fwd 214:3,213:3" "G.g_h2.dgrad 214:3" "D2.fwd 210:2"; do
  set -- $sc
  timeout -k 10 120 python benchmarks/kprobe.py --shape "$1" --cfgs "$2" --reps 20 2>&1 | grep -v amdgpu.ids || exit 1
done
