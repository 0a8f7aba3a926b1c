#!/bin/bash
# kernel-trace step profile of one bench configuration: $1 = tag, remaining args -> bench.py
mkdir -p gpurun_out
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- python3 bench.py "$@" \
  > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
tail -1 gpurun_out/prof_$tag.log
