#!/bin/bash
# round 5, call H: kernel trace of the default (eager) 64x64 step + per-kernel PMC table
mkdir -p gpurun_out
bash scripts/gpu_prof_cfg.sh p64 --steps 20 --warmup 5 || exit 1
python3 scripts/prof_summary.py $(find gpurun_out/prof_p64 -name '*.db' | head -1) --steps 20 > gpurun_out/step_profile_r5.txt 2>&1 || true
python3 scripts/step_queues.py $(find gpurun_out/prof_p64 -name '*.db' | head -1) > gpurun_out/step_queues_r5.txt 2>&1 || true
tail -75 gpurun_out/step_profile_r5.txt | head -5
OUT=step_pmc_r5.txt bash scripts/gpu_pmc_step.sh > /dev/null 2>&1 || { echo pmc failed; exit 1; }
head -32 gpurun_out/step_pmc_r5.txt
