#!/bin/bash
# round 5: tile table tuned under the W=8 DDP stand-in vs the shipped (fused-tuned) table, stand-in at W=2/4/8 + W=1 force_ddp, interleaved
set -o pipefail
mkdir -p gpurun_out
T=benchmarks/tuned_tables/tuned_ddp_w8_r5.json
ab=gpurun_out/ab_ddp_table_r5.txt; : > $ab
for r in 1 2; do
  for w in 8 4 2; do
    for t in shipped ddp; do
      if [ $t = ddp ]; then export DCGAN_TUNED_PATH=$T; else unset DCGAN_TUNED_PATH; fi
      x=$(timeout -k 10 150 python3 -m benchmarks.phase_timing --graph 0 --fake_busbw_gbs 150 --fake_world $w 2>/dev/null | grep '^{') || exit 1
      echo "standin W=$w fp32 table=$t $x" >> $ab
    done
  done
  unset DCGAN_TUNED_PATH
done
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_ddp_table_r5.txt'):
    pre, js = l.split('{', 1); d = json.loads('{' + js)
    print(pre.strip(), d['ms_per_step_timed'])
PY
js() { grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for r in 1 2; do
  x=$(timeout -k 10 150 python3 bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "W=1 force_ddp shipped :: $x"
  x=$(DCGAN_TUNED_PATH=$T timeout -k 10 150 python3 bench.py --force_ddp --steps 200 --warmup 20 2>/dev/null | js) || exit 1; echo "W=1 force_ddp ddp-table :: $x"
done | tee -a $ab
