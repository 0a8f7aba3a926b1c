#!/bin/bash
# igemmh vs igemm3 ablations on the big mode-0 / mode-1 GEMMs (timing only: outputs wrong)
mkdir -p gpurun_out
: > gpurun_out/h_ablate.log
for ab in 0 1 2 4 8 12; do
  DCGAN_IGEMM_ABLATE=$ab timeout -k 10 200 python -u benchmarks/bench_kernels.py --batch 128 --reps 8 --top 40 \
    --only D1.fwd --cfgs 4,210,211,213 2>&1 | grep -v amdgpu.ids | sed "s/^/ab=$ab /" >> gpurun_out/h_ablate.log || exit 1
  DCGAN_IGEMM_ABLATE=$ab timeout -k 10 200 python -u benchmarks/bench_kernels.py --batch 128 --reps 8 --top 40 \
    --only G.g_h3.fwd --cfgs 4,211,213 2>&1 | grep -v amdgpu.ids | sed "s/^/ab=$ab /" >> gpurun_out/h_ablate.log || exit 1
done
cut -c1-400 gpurun_out/h_ablate.log
