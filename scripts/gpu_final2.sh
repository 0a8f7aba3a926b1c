#!/bin/bash
# final numbers of the final tree: smoke, every config family, the driver's form vs 200/20 x3
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { cat gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
./scripts/gpu_configs.sh || exit 1
for i in 1 2 3; do for f in "--steps 20 --warmup 5" "--steps 200 --warmup 20"; do
  r=$(timeout -k 10 120 python bench.py --gpus 1 $f 2>/dev/null) || exit 1
  echo "[$f] $(echo "$r" | python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/bench_final2.txt
