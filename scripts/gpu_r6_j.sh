#!/bin/bash
# round 6: halo K loop -- isolated per-layer sweep at 64x64 (D dgrads, forward convs / deconvs;
# igemm3 21x vs halo 3xx), then the in-situ tuner at 256x256 fp16 over the four largest deconv
# entries with the halo configs as candidates (study table)
mkdir -p gpurun_out
{ timeout -k 10 300 python -u benchmarks/bench_kernels.py --size 64 --batch 128 --only dgrad2B --cfgs 21,20,3 --reps 10 || exit 1
  timeout -k 10 300 python -u benchmarks/bench_kernels.py --size 64 --batch 128 --only G.g_h --cfgs 21,20,3 --reps 10 || exit 1
} > gpurun_out/bench_halo64_r6.txt 2>&1 || { tail -20 gpurun_out/bench_halo64_r6.txt; exit 1; }
grep -v "^\s*$" gpurun_out/bench_halo64_r6.txt | tail -40
timeout -k 10 700 python -u -m benchmarks.tune_insitu --output_size 256 --batch 512 --dtype fp16 --steps 30 --warmup 5 \
  --keys "1,512,32,32,256,64,64,128|1,512,64,64,128,128,128,64|1,1024,32,32,256,64,64,128|1,1024,64,64,128,128,128,64" \
  --extra_cfgs 300,303,304,305,310,313,314,315 --out gpurun_out/tuned_halo256_r6.json > gpurun_out/tune_halo256_r6.txt 2>&1 || { tail -20 gpurun_out/tune_halo256_r6.txt; exit 1; }
grep -v "^\s*$" gpurun_out/tune_halo256_r6.txt | tail -45
