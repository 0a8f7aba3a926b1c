#!/bin/bash
# Full GPU validation: kernel/engine tests, a rocprofv3 kernel-trace profile and the bench.
# Stops at the first GPU fault / abort / timeout (any rc other than 0 or a plain pytest failure).
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python bench.py --steps 20 --warmup 3 > gpurun_out/prof3.log 2>&1 || { tail -20 gpurun_out/prof3.log; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
