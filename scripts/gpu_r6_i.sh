#!/bin/bash
# round 6: step PMC table (current tree), then the in-situ tuner over the 64x64 deconv entries with
# the halo configs as candidates (study table, not written to ops/)
mkdir -p gpurun_out
OUT=step_pmc_r6.txt bash ./scripts/gpu_pmc_step.sh > /dev/null || exit 1
head -30 gpurun_out/step_pmc_r6.txt
timeout -k 10 700 python -u -m benchmarks.tune_insitu --steps 100 --keys "1,128,4,4,512,8,8,256|1,128,8,8,256,16,16,128|1,128,16,16,128,32,32,64|1,256,4,4,512,8,8,256|1,256,8,8,256,16,16,128|1,256,16,16,128,32,32,64" --extra_cfgs 300,303,304,305,310,313,314,315 --out gpurun_out/tuned_halo64_r6.json > gpurun_out/tune_halo64_r6.txt 2>&1 || { tail -20 gpurun_out/tune_halo64_r6.txt; exit 1; }
tail -30 gpurun_out/tune_halo64_r6.txt
