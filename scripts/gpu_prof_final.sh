#!/bin/bash
# final tree: kernel-trace step profile + the two PMC passes of the 64x64 step
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/prof_final.log 2>&1 || { tail -20 gpurun_out/prof_final.log; exit 1; }
python3 scripts/prof_summary.py $(find gpurun_out/prof_final -name '*.db' | head -1) --steps 20 > gpurun_out/step_profile_final.txt && head -5 gpurun_out/step_profile_final.txt
OUT=step_pmc_final.txt ./scripts/gpu_pmc_step.sh
