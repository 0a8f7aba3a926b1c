#!/bin/bash
# igemm3 ablations (timing only, outputs wrong): bit0 no A fetch, bit1 no B fetch, bit2 no LDS
# fragment reads / MFMAs, bit3 no LDS-DMA issue
mkdir -p gpurun_out; : > gpurun_out/ablate.log
for ab in 0 3 4 8 12; do
  for only in D1.fwd D1.dgrad2B G.g_h3.fwd; do
    DCGAN_IGEMM_ABLATE=$ab timeout -k 10 120 python -u benchmarks/bench_kernels.py --batch 128 --reps 10 --only $only \
      2>/dev/null | grep -v amdgpu.ids | sed "s/^/ab=$ab /" | cut -c1-200 >> gpurun_out/ablate.log || exit 1
  done
done
cat gpurun_out/ablate.log
