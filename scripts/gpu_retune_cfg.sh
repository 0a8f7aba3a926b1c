#!/bin/bash
# In-situ retune (sibling tiles, one pass) of another config, then A/B of the result vs the committed
# table on that config's bench, interleaved x2. $1 = tune_insitu args, $2 = bench.py args, $3 = tag
mkdir -p gpurun_out
tag=$3
timeout -k 10 840 python -u -m benchmarks.tune_insitu --tiles --passes 1 $1 --out gpurun_out/tuned_$tag.json > gpurun_out/retune_$tag.txt 2>&1 || { tail -20 gpurun_out/retune_$tag.txt; exit 1; }
grep -E "keep|incumbent|pass" gpurun_out/retune_$tag.txt
python3 -c "import json; json.dump(json.load(open('gpurun_out/tuned_$tag.json'))['table'], open('gpurun_out/tuned_${tag}_table.json', 'w'), indent=1)" || exit 1
for i in 1 2; do for t in new old; do
  if [ $t = new ]; then p=gpurun_out/tuned_${tag}_table.json; else p=distributed_tensorflow_for_dcgan_amd/ops/igemm_tuned.json; fi
  r=$(DCGAN_TUNED_PATH=$p timeout -k 10 300 python bench.py $2 2>/dev/null) || exit 1
  echo "[$t] $(echo "$r" | python3 -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][0]); print(d["value"], d["ms_per_step"])')"
done; done | tee gpurun_out/ab_retune_$tag.txt
