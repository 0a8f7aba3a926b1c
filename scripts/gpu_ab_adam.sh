#!/bin/bash
# A/B: Adam(D) beside G's backward on the D stream (DCGAN_EARLY_ADAM_D=1) vs one fused Adam after the join
mkdir -p gpurun_out
: > gpurun_out/ab_adam.log
for rep in 1 2 3; do
  for v in 1 0; do
    echo "[DCGAN_EARLY_ADAM_D=$v]" >> gpurun_out/ab_adam.log
    DCGAN_EARLY_ADAM_D=$v timeout -k 10 120 python bench.py --steps 200 --warmup 20 >> gpurun_out/ab_adam.log 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json, re, collections
d = collections.defaultdict(list); k = None
for line in open("gpurun_out/ab_adam.log"):
    m = re.match(r"\[(.*)\]", line)
    if m: k = m.group(1); continue
    if line.startswith("{"): d[k].append(json.loads(line)["ms_per_step"])
for k, v in d.items(): print(k, ["%.4f" % x for x in v])
PY
