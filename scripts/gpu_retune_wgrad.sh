#!/bin/bash
# Re-run the per-layer igemm tuner (writes ops/igemm_tuned.json on the box), then A/B the step
# with the new table vs the previous one (copied to /tmp), then copy the new table back.
mkdir -p gpurun_out/tuned
T=distributed_tensorflow_for_dcgan_amd/ops/igemm_tuned.json
cp $T /tmp/tuned_prev.json
timeout -k 10 600 python benchmarks/bench_wgrad.py --batch 128 --write > gpurun_out/ktune.log 2>&1 || { tail -20 gpurun_out/ktune.log; exit 1; }
cp $T gpurun_out/tuned/igemm_tuned.json
cat gpurun_out/ktune.log | cut -c1-150
: > gpurun_out/ab.log
for i in 1 2 3; do
  for v in "X=0" "DCGAN_TUNED_PATH=/tmp/tuned_prev.json"; do
    env $v timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/ab1.log 2>&1 || { tail gpurun_out/ab1.log; exit 1; }
    echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab1.log)" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
