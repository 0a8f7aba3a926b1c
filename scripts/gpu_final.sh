#!/bin/bash
# final validation: the whole GPU suite, smoke, then the driver's form vs 200/20 interleaved x3
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { cat gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
for i in 1 2 3; do for f in "--steps 20 --warmup 5" "--steps 200 --warmup 20"; do
  r=$(timeout -k 10 120 python bench.py --gpus 1 $f 2>/dev/null) || exit 1
  echo "[$f] $(echo "$r" | python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/bench_final.txt
