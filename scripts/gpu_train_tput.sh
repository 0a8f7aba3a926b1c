#!/bin/bash
# Real-training throughput next to bench.py: loader alone, image_train.py on synthetic data and
# on float64 TFRecords (reference format), bs=128, log line every step (async loss ring).
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_loader.py --threads 16 --seconds 8 > gpurun_out/loader.json 2>/dev/null || exit $?
cat gpurun_out/loader.json
COMMON="--batch_size=128 --max_steps=400 --log_every=1 --save_summaries_secs=100000 --sample_every=0 --save_model_secs=1e9 --nosummaries"
timeout -k 10 300 python -u image_train.py --synthetic $COMMON --checkpoint_dir=/tmp/ck_syn --sample_dir=/tmp/s_syn \
  > gpurun_out/train_syn.log 2>&1 || { tail -20 gpurun_out/train_syn.log; exit 1; }
timeout -k 10 300 python -u image_train.py --data_dir=/tmp/dcgan_loader_bench --shuffle_buffer=2048 $COMMON \
  --checkpoint_dir=/tmp/ck_tfr --sample_dir=/tmp/s_tfr > gpurun_out/train_tfr.log 2>&1 || { tail -20 gpurun_out/train_tfr.log; exit 1; }
timeout -k 10 120 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_ref.json 2>/dev/null || exit 1
python - <<'PY'
import json, re, statistics
def rate(path):
    v = [float(m.group(1)) for m in re.finditer(r"images/sec: ([0-9.]+)", open(path).read())]
    v = v[len(v) // 2:]
    return statistics.median(v) if v else 0.0
b = json.loads(open("gpurun_out/bench_ref.json").read().strip().splitlines()[-1])["value"]
s, t = rate("gpurun_out/train_syn.log"), rate("gpurun_out/train_tfr.log")
out = {"bench_img_s": b, "image_train_synthetic_img_s": round(s, 1), "synthetic_vs_bench": round(s / b, 3),
       "image_train_tfrecord_img_s": round(t, 1), "tfrecord_vs_bench": round(t / b, 3)}
print(json.dumps(out))
json.dump(out, open("gpurun_out/train_tput.json", "w"))
PY
