#!/bin/bash
# generic A/B: bash scripts/gpu_ab.sh "ENV1=.." "ENV2=.." ...  (3 rounds of bench.py each)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
for i in 1 2 3; do
for env in "$@"; do
echo "[$env]" >> gpurun_out/ab.log
env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 >> gpurun_out/ab.log 2>&1 || exit 1
done; done
python - <<'PY' >> gpurun_out/ab.log
import json, collections
d = collections.defaultdict(list); cur = None
for l in open("gpurun_out/ab.log"):
    if l.startswith("["): cur = l.strip()
    elif l.startswith("{"): d[cur].append(json.loads(l)["ms_per_step"])
for k, v in d.items(): print("SUMMARY", k, "min %.4f mean %.4f" % (min(v), sum(v) / len(v)))
PY
