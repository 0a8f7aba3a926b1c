#!/bin/bash
# Timing-only ablation of the igemm3 feed: normal / no A loads / no B loads / no loads.
mkdir -p gpurun_out; : > gpurun_out/ablate.log
for shape_cfg in "D1.fwd 210:1,200:1,215:1" "D3.fwd 213:3,210:4" "G.g_h1.dgrad 213:6" "D2.fwd 210:2"; do
  set -- $shape_cfg
  for ab in 0 1 2 3; do
    echo "== $1 ablate=$ab" >> gpurun_out/ablate.log
    DCGAN_IGEMM_ABLATE=$ab timeout -k 10 120 python benchmarks/kprobe.py --shape "$1" --cfgs "$2" --reps 20 >> gpurun_out/ablate.log 2>&1 || exit 1
  done
done
cat gpurun_out/ablate.log | grep -v amdgpu.ids
