#!/bin/bash
# A/B of im2col rows per workgroup (4 vs 8): exactness test, kernel time under rocprofv3, step time.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "im2col or engine_step or d0" --timeout 120 --timeout-method thread > gpurun_out/ab_im2col_tests.log 2>&1 || { tail -30 gpurun_out/ab_im2col_tests.log; exit 1; }
for r in 4 8; do
  DCGAN_IM2COL_ROWS=$r timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/abim$r -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/abim$r.log 2>&1 || exit 1
done
for i in 1 2; do for r in 4 8; do
  echo "rows=$r $(DCGAN_IM2COL_ROWS=$r timeout -k 10 180 python3 bench.py --steps 300 --warmup 30 | tail -1)" >> gpurun_out/ab_im2col_bench.log || exit 1
done; done
find gpurun_out/abim4 gpurun_out/abim8 -name '*stats*' | head
