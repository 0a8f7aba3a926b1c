#!/bin/bash
# LDS fill-path microbenchmark, sampler throughput (64x64 bf16, B = 128 / 512), then an in-situ retune pass with sibling tiles
mkdir -p gpurun_out
timeout -k 10 120 ./benchmarks/study/ldsdma_bw > gpurun_out/ldsdma_bw.txt 2>&1 || { cat gpurun_out/ldsdma_bw.txt; exit 1; }
cat gpurun_out/ldsdma_bw.txt
timeout -k 10 180 python -u benchmarks/bench_sampler.py --sizes 128,512 > gpurun_out/bench_sampler.txt 2>&1 || { tail -20 gpurun_out/bench_sampler.txt; exit 1; }
grep '^{' gpurun_out/bench_sampler.txt
./scripts/gpu_retune.sh --tiles
