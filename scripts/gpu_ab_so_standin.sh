#!/bin/bash
# A/B of two builds (tree vs ab_old/: package + bench.py + benchmarks/) on the DDP step: the
# RCCL-like stand-in at W=8 / 2 (fp32 wire, 150 GB/s, eager) and --force_ddp, interleaved x3;
# $1 = pytest -k expr run first on the new build
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_engine.py tests/test_hip_ddp.py -k "$1" -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/ab_so_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab_so_tests.log; [ $rc -eq 0 ] || exit $rc
st() { python3 -c 'import json,sys
for l in sys.stdin:
    l=l.strip()
    if l.startswith("{"):
        d=json.loads(l); print(d.get("value",""), d.get("ms_per_step",""), d.get("ms_per_step_timed",""), json.dumps(d.get("phases_ms","")))'; }
for i in 1 2 3; do for t in new old; do
  d=.; [ $t = old ] && d=ab_old
  for W in 8 2; do
    r=$(cd $d && timeout -k 10 120 python -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --fake_world $W --steps 50 --warmup 20 2>/dev/null) || exit 1
    echo "[$t standin W=$W] $(echo "$r" | st)"
  done
  r=$(cd $d && timeout -k 10 120 python bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null) || exit 1
  echo "[$t force_ddp] $(echo "$r" | st)"
done; done | tee gpurun_out/ab_so_standin.txt
