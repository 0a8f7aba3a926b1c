#!/bin/bash
# round 6 final numbers: every config family, then the driver's exact form vs 200/20 interleaved x3
mkdir -p gpurun_out
./scripts/gpu_configs.sh || exit 1
for i in 1 2 3; do for f in "--steps 20 --warmup 5" "--steps 200 --warmup 20"; do
  r=$(timeout -k 10 120 python bench.py --gpus 1 $f 2>/dev/null) || exit 1
  echo "[$f] $(echo "$r" | python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/bench_driver_form_r6.txt
