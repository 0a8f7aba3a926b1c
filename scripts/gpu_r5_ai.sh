#!/bin/bash
# round 5: adam2 with two float4 sets per thread (DCGAN_ADAM2_U2) -- test + interleaved A/B + kernel time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_hip_engine.py -m gpu -x -q --timeout 240 --timeout-method thread -k "adam or placements" > gpurun_out/gpu_tests_adam2_u2_r5.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_adam2_u2_r5.log; [ $rc -eq 0 ] || exit $rc
ab=gpurun_out/ab_adam2_u2_r5.txt; : > $ab
for r in 1 2 3; do
  for v in 1 0; do
    x=$(DCGAN_ADAM2_U2=$v timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 2>/dev/null | grep '^{') || exit $?
    echo "round $r adam2_u2=$v $x" >> $ab
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_adam2_u2_r5.txt'):
    pre, js = l.split('{', 1); d = json.loads('{' + js)
    print(pre.strip(), round(d['value']), d['ms_per_step'])
PY
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  DCGAN_ADAM2_U2=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_adam_u2_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 > /dev/null 2>&1 || exit $?
  f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_adam_u2_$v -name '*kernel_stats.csv' | head -1)
  echo "u2=$v"; grep -i adam2 "$f" | cut -d, -f1-6
done
