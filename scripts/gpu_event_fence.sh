#!/bin/bash
# cross-stream marks: native events with a device-scope release (DCGAN_EVENT_FENCE=device) vs
# torch events -- bit-identity checks, then the headline A/B at 200/20 and 20/5, and --force_ddp
mkdir -p gpurun_out
DCGAN_EVENT_FENCE=device timeout -k 10 600 python -u -m pytest tests/test_hip_engine.py tests/test_hip_ddp.py -q -x -k "graph or fused or two_ranks" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_fence.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_fence.log; [ $rc -eq 0 ] || exit $rc
./scripts/gpu_ab_vals.sh DCGAN_EVENT_FENCE "torch device" || exit 1
./scripts/gpu_ab_vals.sh DCGAN_EVENT_FENCE "torch device" --steps 20 --warmup 5 || exit 1
for i in 1 2; do for v in torch device; do
  r=$(DCGAN_EVENT_FENCE=$v timeout -k 10 120 python bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null) || exit 1
  echo "[force_ddp $v] $(echo "$r" | python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/ab_fence_ddp.txt
