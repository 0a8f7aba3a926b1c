#!/bin/bash
# D-wgrad mirror: bitwise test + A/B at 128x128 bf16 and 256x256 fp16; 128x128 step timeline;
# then seeded in-situ tuning of the 28x28x1 step
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_multistep.py -k mirror -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/mirror_test.log 2>&1 || { tail -20 gpurun_out/mirror_test.log; exit 1; }
tail -1 gpurun_out/mirror_test.log
for i in 1 2; do for f in 0 1; do
  echo "[DCGAN_D_WGRAD_ON_G=$f] 128"; DCGAN_D_WGRAD_ON_G=$f timeout -k 10 120 python bench.py --steps 50 --warmup 10 --output_size 128 2>/dev/null | cut -c1-200 || exit 1
done; done | tee gpurun_out/ab_mirror.txt
for f in 0 1; do
  echo "[DCGAN_D_WGRAD_ON_G=$f] 256"; DCGAN_D_WGRAD_ON_G=$f timeout -k 10 200 python bench.py --steps 8 --warmup 3 --output_size 256 --batch_size 512 --dtype fp16 2>/dev/null | cut -c1-200 || exit 1
done | tee -a gpurun_out/ab_mirror.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_128 -o run -- python3 bench.py --steps 10 --warmup 3 --output_size 128 \
  > gpurun_out/prof_128.log 2>&1 || { tail -20 gpurun_out/prof_128.log; exit 1; }
bash scripts/gpu_tune_insitu.sh s28 --output_size 28 --c_dim 1 --batch 128 --steps 60 --warmup 10 --seed --passes 1
