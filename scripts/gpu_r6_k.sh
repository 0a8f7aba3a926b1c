#!/bin/bash
# round 6: linear forward with k-quarter waves (test + A/B vs ab_old), then the sharded-DDP
# validation (scripts/gpu_r6_g.sh)
mkdir -p gpurun_out
./scripts/gpu_ab_so.sh "linear or philox" || exit 1
./scripts/gpu_r6_g.sh
