#!/bin/bash
# wgrad3 bring-up: kernel numerics first (stop on failure), per-layer tuning (writes
# ops/igemm_tuned.json, copied to gpurun_out/tuned/), engine tests, bench + rocprofv3 profile.
mkdir -p gpurun_out/tuned
step() {  # step <name> <timeout> <cmd...>: stop the script on any failure (faults included)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step w3test 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "wgrad" --timeout 120 --timeout-method thread
TAILN=12 step wbench 600 python benchmarks/bench_wgrad.py --batch 128 --write
cp distributed_tensorflow_for_dcgan_amd/ops/igemm_tuned.json gpurun_out/tuned/
step engine 600 python -u -m pytest tests/test_hip_engine.py tests/test_hip_ddp.py -x -q -m gpu --timeout 300 --timeout-method thread
step bench 300 python bench.py --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof4
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run -- python bench.py --steps 20 --warmup 3
