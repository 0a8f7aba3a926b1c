#!/bin/bash
# round 5: G weight-gradient placements (DCGAN_GW_PLACE), timeline + interleaved bench A/B
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/tail_timeline_place_r5.txt; : > $out
for p in ssss sasa; do
  timeout -k 10 120 python3 -u benchmarks/study/tail_timeline.py --place $p >> $out 2>&1 || exit $?
done
ab=gpurun_out/ab_gw_place_r5.txt; : > $ab
for r in 1 2 3; do
  for p in ddcc ssss aaaa sssc sasa ssdd; do
    x=$(DCGAN_GW_PLACE=$p timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | grep '^{') || exit $?
    echo "round $r place=$p $x" >> $ab
  done
done
grep -v amdgpu.ids $out
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_gw_place_r5.txt'):
    pre, js = l.split('{', 1); d = json.loads('{' + js)
    print(pre.strip(), round(d['value']), d['ms_per_step'])
PY
