#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -q -m gpu -x -k igemm3 > gpurun_out/k.log 2>&1 || { tail -30 gpurun_out/k.log; exit 1; }
tail -1 gpurun_out/k.log
for sc in "D1.dgradB 103:1,215:1,213:1,205:1" "D1.dgrad2B 101:1,213:1,210:1,211:1" "G.g_h3.fwd 103:1,215:1,213:1" "D2.dgradB 103:1,215:1,214:1" "G.g_h1.fwd 214:3,214:2"; do
  set -- $sc
  timeout -k 10 120 python benchmarks/kprobe.py --shape "$1" --cfgs "$2" --reps 20 2>&1 | grep -v amdgpu.ids || exit 1
done
