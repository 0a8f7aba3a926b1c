#!/bin/bash
# A/B of env-toggled engine variants (interleaved bench runs), then a rocprofv3 step profile.
# usage: gpu_abprof.sh "ENV=1" [profdir]
mkdir -p gpurun_out; : > gpurun_out/ab.log
for i in 1 2 3; do
  for v in "X=0" "$1"; do
    env $v timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/ab1.log 2>&1 || { tail gpurun_out/ab1.log; exit 1; }
    echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab1.log)" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
P=${2:-prof5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/$P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$P -o run -- python bench.py --steps 20 --warmup 3 > gpurun_out/$P.log 2>&1 || { tail -20 gpurun_out/$P.log; exit 1; }
echo prof ok
