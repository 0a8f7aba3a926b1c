#!/bin/bash
# A/B of one engine switch: scripts/gpu_ab_env.sh VAR "v1 v2 .." [reps]  (bench.py, 200 timed steps each)
VAR=$1; VALS=$2; REPS=${3:-3}
mkdir -p gpurun_out
log=gpurun_out/ab_$VAR.log; : > $log
for rep in $(seq $REPS); do
  for v in $VALS; do
    echo "[$VAR=$v]" >> $log
    env $VAR=$v timeout -k 10 120 python bench.py --steps 200 --warmup 20 >> $log 2>/dev/null || exit 1
  done
done
python - "$log" <<'PY'
import json, re, sys, collections
d = collections.defaultdict(list); k = None
for line in open(sys.argv[1]):
    m = re.match(r"\[(.*)\]", line)
    if m: k = m.group(1); continue
    if line.startswith("{"): d[k].append(json.loads(line)["ms_per_step"])
for k, v in d.items(): print(k, ["%.4f" % x for x in v], "min %.4f" % min(v))
PY
