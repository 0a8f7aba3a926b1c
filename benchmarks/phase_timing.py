"""Per-phase GPU timeline of the training step (1 GPU), and the DDP schedules with emulated
collectives: where the D chain and the G chain end, i.e. when each DDP collective can start
(hip_engine.py ``_run_step``), and how much of each collective's latency a schedule hides.

    python -m benchmarks.phase_timing [--batch_size 128] [--steps 50]
    python -m benchmarks.phase_timing --schedule ddp --fake_busbw_gbs 300      (one-graph DDP)
    python -m benchmarks.phase_timing --fake_comm_us 150,60,20                 (segmented DDP)
"""
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
    contention is modelled). Capturable: the "ddp" schedule records it inside its graph."""

    def __init__(self, us, cycles_per_us, numel=0):
        self.us = float(us)
        self.cycles = int(us * cycles_per_us)
        self.numel = numel

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


def ring_us(numel: int, busbw_gbs: float, lat_us: float, world: int, esize: int = 4) -> float:
    """Ring all-reduce time model: latency + 2 (W-1)/W x bytes / bus bandwidth."""
    return lat_us + 2.0 * (world - 1) / world * numel * esize / (busbw_gbs * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--schedule", default="concurrent", choices=["concurrent", "serial", "ddp"])
    ap.add_argument("--fake_comm_us", default="", help="concurrent: G,Dtop,Drest all-reduce latencies (us)")
    ap.add_argument("--fake_busbw_gbs", type=float, default=0.0,
                    help="emulate every bucket with the ring model at this bus bandwidth (GB/s)")
    ap.add_argument("--fake_lat_us", type=float, default=10.0)
    ap.add_argument("--fake_world", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    ddp = a.schedule != "concurrent" or bool(a.fake_comm_us) or a.fake_busbw_gbs > 0
    eng = HipEngine(cfg, a.batch_size, dev, ddp=ddp, schedule=a.schedule if ddp else None)
    if a.schedule in ("concurrent", "serial"):
        eng.enable_timing()  # the segmented schedules, Adam(G) / Adam(D) apart
    cpu = _cycles_per_us() if ddp else 0.0
    comm = {}
    if ddp:
        # collective call points of DDP on a comm stream; the update program is rebuilt for W=2
        # (Adam scales the un-reduced gradients by 1/2: only timing and stream order are emulated)
        eng.world = 2
        eng._build_updates()
        eng._ensure_comm()

        def fake(name, numel, us=None):
            if us is None:
                us = ring_us(numel, a.fake_busbw_gbs, a.fake_lat_us, a.fake_world) if a.fake_busbw_gbs > 0 else 0.0
            comm[name] = round(us, 1)
            return FakeReducer(us, cpu, numel)

        gd, gg = eng.grad_d.flat, eng.grad_g.flat
        o = eng._d_top_off
        us3 = [float(x) for x in a.fake_comm_us.split(",")] if a.fake_comm_us else [None] * 3
        eng._ar_g = fake("g", gg.numel(), us3[0])
        eng._ar_dtop = fake("dtop", gd.numel() - o, us3[1])
        eng._ar_drest = fake("drest", o, us3[2])
        if a.schedule == "ddp":
            eng._ar_gparts = [fake("g[%d:%d]" % (lo, hi), hi - lo) for _, lo, hi in eng._g_cuts]
    eng.set_synthetic_batch(torch.rand(a.batch_size, 64, 64, 3, device=dev) * 2 - 1)
    for _ in range(a.warmup):
        eng.train_step()
    acc = {}
    if eng._timing:
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
    print(json.dumps({"schedule": eng._schedule(), "graph": eng.graph_enabled, "fake_comm_us": comm,
                      "ms_per_step_timed": round(ms, 4), "phases_ms": {k: round(v, 4) for k, v in acc.items()}}))


if __name__ == "__main__":
    main()
