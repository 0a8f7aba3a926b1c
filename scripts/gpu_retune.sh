#!/bin/bash
# Re-tune the tile table in situ (whole-step time, current tree) and A/B the result against the
# committed table, interleaved x3 at the driver's form and at 200/20. $1 = extra tune_insitu args
mkdir -p gpurun_out
timeout -k 10 840 python -u -m benchmarks.tune_insitu --passes 1 --steps 150 --warmup 20 --out gpurun_out/tuned_retune.json $1 \
  > gpurun_out/retune.txt 2>&1 || { tail -20 gpurun_out/retune.txt; exit 1; }
grep -E "keep|incumbent|pass" gpurun_out/retune.txt
python3 -c "import json; json.dump(json.load(open('gpurun_out/tuned_retune.json'))['table'], open('gpurun_out/tuned_retune_table.json', 'w'), indent=1)" || exit 1
for i in 1 2 3; do for t in new old; do
  if [ $t = new ]; then p=gpurun_out/tuned_retune_table.json; else p=distributed_tensorflow_for_dcgan_amd/ops/igemm_tuned.json; fi
  for f in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    r=$(DCGAN_TUNED_PATH=$p timeout -k 10 120 python bench.py $f 2>/dev/null) || exit 1
    echo "[$t $f] $(echo "$r" | python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])')"
  done
done; done | tee gpurun_out/ab_retune.txt
