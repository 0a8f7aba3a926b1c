"""Sampling (inference) throughput of the HIP engine: G's forward with inference-mode BN (the
moving averages), the path of ``image_train.py --visualize`` / the trainer's sample grids
(reference: ``/root/reference/distriubted_model.py:131-153`` sampler, ``image_train.py:176-190``).

One JSON line per batch size: images/sec of the recorded sampler Program replayed back to back
(z copied in once; each replay regenerates the whole batch), random-init weights after a few
training steps (so the moving averages are populated).

    python benchmarks/bench_sampler.py [--sizes 128,512] [--output_size 64] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="128,512")
    ap.add_argument("--output_size", type=int, default=64)
    ap.add_argument("--c_dim", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig(output_size=a.output_size, c_dim=a.c_dim)
    for B in [int(s) for s in a.sizes.split(",") if s]:
        eng = HipEngine(cfg, B, dev, graph=False, dtype=a.dtype)
        real = torch.rand(B, cfg.output_size, cfg.output_size, cfg.c_dim, device=dev) * 2 - 1
        eng.set_synthetic_batch(real)
        for _ in range(3):  # populate the BN moving averages
            eng.train_step()
        z = torch.rand(B, cfg.z_dim, device=dev) * 2 - 1
        img = eng.sampler(z)  # builds the sampler Program, sets the debias factor and z
        assert img.shape == (B, cfg.output_size, cfg.output_size, cfg.c_dim) and bool(torch.isfinite(img).all())
        for _ in range(a.warmup):
            H.run(eng.progS)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            H.run(eng.progS)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        print(json.dumps({"metric": "sampler images/sec (G forward, inference BN), %dx%dx%d"
                          % (cfg.output_size, cfg.output_size, cfg.c_dim),
                          "batch": B, "dtype": a.dtype, "value": round(B / dt, 1), "ms_per_batch": round(dt * 1e3, 4),
                          "launches": sum(1 for i in range(eng.progS.size())
                                          if eng.progS.op_info(i)[2] == eng.ext.OP_LAUNCH)}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
