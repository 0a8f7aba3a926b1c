"""Per-phase GPU timeline of the training step (1 GPU): where the D chain and the G chain of
the concurrent schedule end, i.e. when each DDP collective can start (hip_engine.py
``_run_step``). ``python -m benchmarks.phase_timing [--batch_size 128] [--steps 50]``."""
import argparse
import json
import time

import torch

from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig


class FakeReducer:
    """Stand-in for parallel.dist.GradAllReducer on ONE GPU: occupies the comm stream for a
    given time (a spinning kernel), at the same points of the schedule as the real
    all-reduce, to see which schedule hides which collective latency (no bandwidth
    contention is modelled)."""

    def __init__(self, us, cycles_per_us):
        self.cycles = int(us * cycles_per_us)

    def issue(self):  # on the comm stream (the engine's executor orders it after the producers)
        if self.cycles > 0:
            torch.cuda._sleep(self.cycles)


def _cycles_per_us():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    e0.record()
    torch.cuda._sleep(1000000)
    e1.record()
    e1.synchronize()
    return 1000000 / (e0.elapsed_time(e1) * 1000.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--fake_comm_us", default="", help="G,Dtop,Drest all-reduce latencies (us)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    eng = HipEngine(cfg, a.batch_size, dev)
    eng.enable_timing()  # the segmented "concurrent" schedule, Adam(G) / Adam(D) apart
    if a.fake_comm_us:
        g_us, top_us, rest_us = (float(x) for x in a.fake_comm_us.split(","))
        cpu = _cycles_per_us()
        # collective call points of DDP on a comm stream; the update program is rebuilt for W=2
        # (Adam scales the un-reduced gradients by 1/2: only timing and stream order are emulated)
        eng.world = 2
        eng._build_updates()  # the update program a real W=2 build runs (split Adam(G) / Adam(D))
        eng.comm_stream = torch.cuda.Stream(device=dev)
        eng._ar_g, eng._ar_dtop, eng._ar_drest = (FakeReducer(u, cpu) for u in (g_us, top_us, rest_us))
    eng.set_synthetic_batch(torch.rand(a.batch_size, 64, 64, 3, device=dev) * 2 - 1)
    for _ in range(a.warmup):
        eng.train_step()
    acc = {}
    for _ in range(a.steps):
        eng.train_step()
        for k, v in eng.phase_times().items():
            acc[k] = acc.get(k, 0.0) + v / a.steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.train_step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    print(json.dumps({"schedule": eng._schedule(), "fake_comm_us": a.fake_comm_us, "ms_per_step_timed": round(ms, 4),
                      "phases_ms": {k: round(v, 4) for k, v in acc.items()}}))


if __name__ == "__main__":
    main()
