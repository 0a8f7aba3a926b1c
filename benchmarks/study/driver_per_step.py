#!/usr/bin/env python3
"""Per-step anatomy of the driver's bench form (``bench.py --gpus 1 --steps K --warmup W``).

Runs the same engine, the same warmup, the same sync/barrier brackets as bench.py, and records
a HIP event on the main stream at every step boundary (timed steps AND warmup) plus the host
time each ``train_step()`` call took to issue. Prints, per step: GPU ms between consecutive
boundaries, host issue ms, and the host-ahead margin (how far the host was ahead of the GPU when
it issued the step's first launch). The first timed step's GPU time vs the steady state tells a
one-time cost from a clock ramp; the host column tells whether the GPU starves on the issue.

Events cost a few us each; one per step does not change the step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--repeat", type=int, default=3, help="timed blocks, each after sync+barrier")
    p.add_argument("--batch_size", type=int, default=128)
    p.add_argument("--output_size", type=int, default=64)
    p.add_argument("--graph", type=int, default=0)
    a = p.parse_args()
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    from distributed_tensorflow_for_dcgan_amd.engine.factory import build_engine
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    D.init_distributed(1, 0, dev)
    cfg = DCGANConfig(output_size=a.output_size)
    eng = build_engine(cfg, a.batch_size, dev, engine="hip", dtype="bf16", graph=bool(a.graph))
    gen = torch.Generator(device="cpu").manual_seed(1)
    eng.set_synthetic_batch((torch.rand(a.batch_size, cfg.output_size, cfg.output_size, 3, generator=gen) * 2 - 1).to(dev))
    cs = torch.cuda.current_stream()

    def block(n, label):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        host = []
        torch.cuda.synchronize()
        D.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        evs[0].record(cs)
        for i in range(n):
            h = time.perf_counter()
            eng.train_step()
            evs[i + 1].record(cs)
            host.append((time.perf_counter() - h) * 1e3)
        torch.cuda.synchronize()
        D.barrier()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        gpu = [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]
        tot = evs[0].elapsed_time(evs[-1])
        print("%s: wall %.3f ms (%.4f ms/step), event span %.3f ms, sum(host issue) %.3f ms"
              % (label, wall, wall / n, tot, sum(host)))
        print("   step  gpu_ms  host_ms")
        for i in range(n):
            print("   %4d  %6.4f  %6.4f" % (i, gpu[i], host[i]))
        return {"label": label, "wall_ms": wall, "event_ms": tot, "gpu": gpu, "host": host}

    out = [block(a.warmup, "warmup")]
    for r in range(a.repeat):
        out.append(block(a.steps, "timed#%d" % r))
    # steady state reference: a long block
    out.append(block(200, "long200"))
    print(json.dumps({"summary": [(o["label"], round(o["wall_ms"], 3), round(o["event_ms"], 3)) for o in out]}))


if __name__ == "__main__":
    main()
