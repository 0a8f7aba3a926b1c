#!/bin/bash
# A/B: number of trailing G layers whose weight gradient runs on the side stream (DCGAN_G_WGRAD_SIDE)
mkdir -p gpurun_out
: > gpurun_out/ab_side.log
for rep in 1 2; do
  for v in 0 1 2 3; do
    echo "[DCGAN_G_WGRAD_SIDE=$v]" >> gpurun_out/ab_side.log
    DCGAN_G_WGRAD_SIDE=$v timeout -k 10 120 python bench.py --steps 200 --warmup 20 >> gpurun_out/ab_side.log 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json, re, collections
d = collections.defaultdict(list); k = None
for line in open("gpurun_out/ab_side.log"):
    m = re.match(r"\[(.*)\]", line)
    if m: k = m.group(1); continue
    if line.startswith("{"): d[k].append(json.loads(line)["ms_per_step"])
for k, v in d.items(): print(k, ["%.4f" % x for x in v])
PY
