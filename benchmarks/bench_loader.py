#!/usr/bin/env python3
"""Input-pipeline throughput of the native TFRecord loader (the reference's 16-thread
``shuffle_batch`` queue, image_input.py:77-84), on the reference's own record format:
tf.train.Example protos whose ``image_raw`` is a raw little-endian float64 [64,64,3] image.

Writes ``--records`` such records (``--files`` files, CRC32C-framed, data/tfrecord.py) once,
then times ``Loader.next_batch`` -- CRC check, Example parse, float64 -> training-dtype decode,
shuffle-pool draw -- into a pinned host buffer (the H2D copy of the training pipeline is async
on a side stream and is not part of this number). Prints one JSON line.

    python benchmarks/bench_loader.py [--threads 16] [--out_dtype bf16] [--seconds 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_tensorflow_for_dcgan_amd.data import native  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.data import tfrecord as TR  # noqa: E402


def make_dataset(d: str, records: int, files: int, shape, seed: int = 0) -> list:
    os.makedirs(d, exist_ok=True)
    paths = [os.path.join(d, "train-%05d-of-%05d.tfrecord" % (i, files)) for i in range(files)]
    want = -(-records // files)
    if all(os.path.exists(p) and native.ext().count_records(p) == want for p in paths):
        return paths
    rng = np.random.default_rng(seed)
    for p in paths:
        recs = [TR.encode_image_example(rng.uniform(-1, 1, shape), "float64") for _ in range(want)]
        native.ext().write_records(p, recs)
    return paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/dcgan_loader_bench")
    ap.add_argument("--records", type=int, default=4096)
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--shuffle_buffer", type=int, default=1024)
    ap.add_argument("--out_dtype", default="bf16", choices=["f32", "bf16", "f16"])
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--verify_crc", type=int, default=1)
    a = ap.parse_args()
    shape = (a.size, a.size, 3)
    t0 = time.time()
    files = make_dataset(a.dir, a.records, a.files, shape)
    gen_s = time.time() - t0
    import torch
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[a.out_dtype]
    pin = torch.cuda.is_available()
    host = torch.empty((a.batch,) + shape, dtype=dt, pin_memory=pin)
    ld = native.ext().Loader(files, "image_raw", a.size, a.size, 3, a.batch, a.shuffle_buffer + 3 * a.batch,
                             a.shuffle_buffer, a.threads, 1, a.out_dtype, "auto", True, bool(a.verify_crc))
    for _ in range(3):  # fill the shuffle pool
        ld.next_batch(host.data_ptr())
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        n += ld.next_batch(host.data_ptr())
    dt_s = time.perf_counter() - t0
    st = ld.stats()
    ld.stop()
    ref = torch.from_numpy(TR.decode_image_example(native.ext().read_records(files[0], True)[0], shape))
    assert torch.isfinite(host.float()).all() and host.float().abs().max() <= 1.0 + 1e-2
    ips = n / dt_s
    print(json.dumps({"metric": "loader images/sec (TFRecord float64 64x64x3 -> %s, pinned host)" % a.out_dtype,
                      "value": round(ips, 1), "unit": "images/sec", "threads": a.threads, "batch": a.batch,
                      "record_bytes": int(np.prod(shape)) * 8, "decode_GBps_f64": round(ips * np.prod(shape) * 8 / 1e9, 2),
                      "cpus": os.cpu_count(), "verify_crc": bool(a.verify_crc), "records_read": st["records"],
                      "epochs": st["epochs"], "dataset_gen_s": round(gen_s, 1),
                      "sample_check": float(ref.abs().max())}), flush=True)


if __name__ == "__main__":
    main()
