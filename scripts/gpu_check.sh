#!/bin/bash
# Engine validation after a step-structure / kernel change: kernel tests (optional filter),
# engine + DDP GPU tests, then the bench.
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: stop the script on any failure (faults included)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -n "$KFILTER" ]; then
  step kern 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "$KFILTER" --timeout 120 --timeout-method thread
fi
step engine 600 python -u -m pytest tests/test_hip_engine.py tests/test_hip_ddp.py -x -q -m gpu --timeout 300 --timeout-method thread
step bench 300 python bench.py --steps 50 --warmup 10
