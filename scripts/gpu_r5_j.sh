#!/bin/bash
# round 5: BN fold bit-exactness + A/B, hoisted igemm3 addressing (new tree vs ab_old/), shared
# engine streams (engine rebuild study)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_hip_kernels.py tests/test_hip_engine.py -k "bn_fold or wgrad_fused_adam or bn_forward_backward or igemm3" \
  > gpurun_out/r5j_tests.log 2>&1 || { tail -30 gpurun_out/r5j_tests.log; exit 1; }
tail -3 gpurun_out/r5j_tests.log
for i in 1 2 3 4; do for f in 0 64 256; do
  r=$(DCGAN_BN_FOLD=$f timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null) || { echo "FAILED $f"; exit 1; }
  echo "DCGAN_BN_FOLD=$f :: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["kernels_per_step"])')"
done; done | tee gpurun_out/ab_bn_fold.txt
for i in 1 2 3 4; do
  r=$(timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null) || exit 1
  echo "hoist(new) :: $(echo "$r" | cut -c1-120)"
  r=$(cd ab_old && timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 2>/dev/null) || exit 1
  echo "old :: $(echo "$r" | cut -c1-120)"
done | tee gpurun_out/ab_hoist.txt
timeout -k 10 200 python3 -u benchmarks/study/engine_rebuild.py --builds 12 > gpurun_out/rebuild_shared.txt 2>&1 || exit 1
tail -1 gpurun_out/rebuild_shared.txt
DCGAN_FRESH_STREAMS=1 timeout -k 10 200 python3 -u benchmarks/study/engine_rebuild.py --builds 12 > gpurun_out/rebuild_fresh.txt 2>&1 || exit 1
tail -1 gpurun_out/rebuild_fresh.txt
