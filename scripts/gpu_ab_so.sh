#!/bin/bash
# A/B of two builds of the extension: the tree (new) vs ab_old/ (git-ignored: a copy of the package
# directory + bench.py with the .so built from the baseline sources -- build the baseline, copy
# distributed_tensorflow_for_dcgan_amd/ and bench.py into ab_old/, rebuild the tree);
# $1 = pytest -k expr run first on the new build; remaining args -> bench.py
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py -k "$1" -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/ab_so_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab_so_tests.log; [ $rc -eq 0 ] || exit $rc
shift
for i in 1 2 3; do
  echo "[new]"; timeout -k 10 120 python bench.py --steps 200 --warmup 20 "$@" 2>/dev/null | cut -c1-200 || exit 1
  echo "[old]"; (cd ab_old && timeout -k 10 120 python bench.py --steps 200 --warmup 20 "$@" 2>/dev/null | cut -c1-200) || exit 1
done | tee gpurun_out/ab_so.txt
