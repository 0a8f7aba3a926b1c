#!/bin/bash
# fused BN finalize: engine parity tests, then A/B bench (fused vs DCGAN_NO_FUSED_FIN=1), alternating
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_engine.py tests/test_hip_kernels.py -q -m gpu -x --timeout 300 \
  --timeout-method thread > gpurun_out/fin_tests.log 2>&1
rc=$?; tail -15 gpurun_out/fin_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ab_fin.txt
for i in 1 2; do
  for v in 0 1; do
    echo "[DCGAN_NO_FUSED_FIN=$v]" >> gpurun_out/ab_fin.txt
    DCGAN_FUSED_FIN=$((1-v)) DCGAN_NO_FUSED_FIN=$v timeout -k 10 120 python bench.py --steps 100 --warmup 20 >> gpurun_out/ab_fin.txt 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json
cur = None; res = {}
for line in open("gpurun_out/ab_fin.txt"):
    if line.startswith("["): cur = line.strip(); continue
    if line.startswith("{"): res.setdefault(cur, []).append(json.loads(line)["ms_per_step"])
for k, v in res.items(): print(k, v)
PY
