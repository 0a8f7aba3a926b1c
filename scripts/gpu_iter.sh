#!/bin/bash
# One GPU iteration: new-kernel tests first (stop on failure), full GPU suite, per-layer tile
# autotune (writes ops/igemm_tuned.json, copied to gpurun_out/tuned/), then the bench with the
# tuned table and a rocprofv3 kernel-trace profile of it.
mkdir -p gpurun_out/tuned
step() {  # step <name> <timeout> <cmd...>: stop the script on any failure (faults included)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step k3 600 python -m pytest tests/test_hip_kernels.py -q -m gpu -x -k "igemm3"
step gpu_tests 900 python -m pytest tests -q -m gpu -x
step kbench 900 python benchmarks/bench_kernels.py --batch 128 --write
cp distributed_tensorflow_for_dcgan_amd/ops/igemm_tuned.json gpurun_out/tuned/
cat gpurun_out/kbench.log
step bench 300 python bench.py --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof3
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python bench.py --steps 20 --warmup 3
