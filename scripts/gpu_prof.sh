#!/bin/bash
# bench (2 runs) + a rocprofv3 kernel-trace of the graph-launched step ($1 = output tag)
mkdir -p gpurun_out
tag=${1:-cur}
for i in 1 2; do timeout -k 10 120 python bench.py --steps 100 --warmup 20 2>/dev/null | cut -c1-200 || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
ls gpurun_out/prof_$tag
