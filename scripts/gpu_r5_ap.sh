#!/bin/bash
# round 5: kernel trace of the final 64x64 step (alt1 weight-gradient placement, re-tuned tiles)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r5c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5c -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_r5c.log 2>&1 || { tail -5 gpurun_out/prof_r5c.log; exit 1; }
db=$(find gpurun_out/prof_r5c -name '*.db' | head -1)
python3 scripts/prof_summary.py "$db" --steps 20 > gpurun_out/step_profile_r5c.txt && head -40 gpurun_out/step_profile_r5c.txt
rm -rf gpurun_out/prof_r5c
