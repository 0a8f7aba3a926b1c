#!/bin/bash
mkdir -p gpurun_out; : > gpurun_out/stamps.log
for sc in "D1.fwd 210:1,215:1,200:1" "D3.fwd 214:3,213:3" "G.g_h2.dgrad 214:3" "G.g_h1.dgrad 215:4"; do
  set -- $sc
  timeout -k 10 120 python benchmarks/kprobe.py --shape "$1" --cfgs "$2" --reps 10 --stamps >> gpurun_out/stamps.log 2>&1 || { cat gpurun_out/stamps.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/stamps.log
