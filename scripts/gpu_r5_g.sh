#!/bin/bash
# round 5, call G: every config (bench_configs), 256x256 fp16 kernel trace, learnability diversity study
mkdir -p gpurun_out
bash scripts/gpu_configs.sh || exit 1
bash scripts/gpu_prof_cfg.sh p256 --steps 5 --warmup 2 --output_size 256 --batch_size 512 --dtype fp16 || exit 1
python3 scripts/prof_summary.py $(find gpurun_out/prof_p256 -name '*.db' | head -1) --steps 5 > gpurun_out/step_profile_256_fp16_r5.txt 2>&1 || true
head -30 gpurun_out/step_profile_256_fp16_r5.txt
timeout -k 10 600 python3 -u benchmarks/study/learn_diag.py one --seeds 4,5,6 --steps 200,400,600 > gpurun_out/learn_diag_r5.txt 2>&1
rc=$?; cat gpurun_out/learn_diag_r5.txt | tail -12; exit $rc
