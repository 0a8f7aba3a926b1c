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
from distributed_tensorflow_for_dcgan_amd.parallel import dist as D


class FakeReducer:
    """Stand-in for parallel.dist.GradAllReducer on ONE GPU, at the same points of the schedule
    as the real all-reduce. ``kind="rccl"`` (default): the RCCL-like copy kernel of
    csrc/hip/comm_emu.hip -- ``nwg`` workgroups (RCCL's channels, one CU each) stream
    2 (W-1)/W x the bucket's bytes through HBM (read the gradient, write a scratch buffer) paced
    to the modelled ring time, so the collective takes CUs and HBM bandwidth from the compute it
    overlaps, as the real one does. ``kind="sleep"``: round 3's single-thread timer
    (``torch.cuda._sleep``: no CU or HBM footprint). Capturable: the "ddp" schedule records it
    inside its graph. With a bf16 wire (esize 2) it also runs the real reducer's two cast copies
    (fp32 gradient -> bf16 wire buffer before the collective, back after it:
    parallel/dist.py GradAllReducer.issue), so the bf16 rows carry their full cost."""

    def __init__(self, us, flat=None, world=8, esize=4, nwg=32, kind="rccl", cycles_per_us=0.0, prefilled=None,
                 wire_copies=True):
        self.us = float(us)
        self.flat = flat
        self.numel = 0 if flat is None else flat.numel()
        self.kind = kind
        self.cycles = int(us * cycles_per_us)
        self.nwg = int(nwg)
        self.bytes = (int(2.0 * (world - 1) / world * self.numel * esize) // 16) * 16
        self.prog = None
        # prefilled: the engine's own bf16 image of the slice (copy-free wire: its casts run inside
        # the step graphs, so the stand-in only streams the image, no copies)
        self.prefilled = prefilled
        self.wire = (torch.empty(self.numel, device=flat.device, dtype=torch.bfloat16)
                     if esize == 2 and flat is not None and prefilled is None and wire_copies else None)
        if kind == "rccl" and self.bytes > 0 and flat is not None:
            from distributed_tensorflow_for_dcgan_amd.ops import hip as H
            payload = prefilled if prefilled is not None else (flat if self.wire is None else self.wire)
            src_bytes = self.numel * payload.element_size()
            # the wire moves up to 2x the payload: read it twice over when the slice is shorter
            self.src = payload if src_bytes >= self.bytes else payload.repeat(-(-self.bytes // src_bytes))
            self.dst = torch.empty(self.bytes // 4, device=flat.device, dtype=torch.float32)
            self.prog = H.ext().Program()
            self.prog.comm_emulate("comm_emu", self.src.data_ptr(), self.dst.data_ptr(), self.bytes, self.us,
                                   self.nwg, 0)

    def issue(self):  # on the comm stream (the engine's executor orders it after the producers)
        if self.wire is not None:
            self.wire.copy_(self.flat)
        if self.kind == "rccl" and self.prog is not None:
            from distributed_tensorflow_for_dcgan_amd.ops import hip as H
            H.run(self.prog)
        elif self.cycles > 0:
            torch.cuda._sleep(self.cycles)
        if self.wire is not None:
            self.flat.copy_(self.wire)

    def accesses(self):  # as the real reducer: the gradient slice is read and written
        if self.flat is None:
            return []
        if self.prefilled is not None:
            return [(self.prefilled.data_ptr(), self.numel * 2, True)]
        out = [(self.flat.data_ptr(), self.numel * self.flat.element_size(), True)]
        if self.wire is not None:
            out.append((self.wire.data_ptr(), self.numel * 2, True))
        return out


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


def standin_engine(cfg, B, dev, schedule="concurrent", ddp=True, graph=False, wire="fp32", busbw_gbs=150.0,
                   lat_us=10.0, world=8, kind="rccl", nwg=32, comm_us="", timing=False, dtype="bf16"):
    """A one-GPU HipEngine running the DDP step with FakeReducer collectives at the real call
    points (the RCCL-like stand-in). Returns (engine, {collective: modelled us})."""
    eng = HipEngine(cfg, B, dev, ddp=ddp, schedule=schedule if ddp else None, allreduce_dtype=wire, graph=graph,
                    dtype=dtype)
    if timing:
        eng.enable_timing()  # the segmented schedules, Adam(G) / Adam(D) apart
    cpu = _cycles_per_us() if ddp and kind == "sleep" else 0.0
    esize = 2 if wire == "bf16" else 4
    comm = {}
    if ddp:
        # collective call points of DDP on a comm stream; the update program is rebuilt for W=2
        # (Adam scales the un-reduced gradients by 1/2: only timing and stream order are emulated)
        eng.world = 2
        if getattr(eng, "_shards", None) is not None:  # sharded update: shards of 1/W, as at W ranks
            eng.shard_world = world
            eng._build_shards()
        eng._build_updates()
        eng._ensure_comm()

        def fake(name, real, us=None):
            flat = real.flat
            if us is None:
                us = ring_us(flat.numel(), busbw_gbs, lat_us, world, esize) if busbw_gbs > 0 else 0.0
            comm[name] = round(us, 1)
            return FakeReducer(us, flat, world, esize, nwg, kind, cpu, prefilled=real.wire if real.prefilled else None)

        if eng._sharded():
            # reduce-scatter: (W-1)/W x 4 B per element, all-gather of the bf16 mirror: (W-1)/W x 2 B
            # (FakeReducer moves 2 (W-1)/W x esize bytes: esize 2 and 1)
            for name, (sr, _, _, _) in eng._shards.items():
                for op, es in (("rs", 2), ("ag", 1)):
                    us = ring_us(sr.grad.numel(), busbw_gbs, lat_us, world, es) if busbw_gbs > 0 else 0.0
                    comm[op + "." + name] = round(us, 1)
                    setattr(sr, op + "_op", FakeReducer(us, sr.grad, world, es, nwg, kind, cpu, wire_copies=False))
            for name, _, _, _ in eng._small:
                setattr(eng, "_ar_" + name, fake(name, getattr(eng, "_ar_" + name)))
            return eng, comm

        us3 = [float(x) for x in comm_us.split(",")] if comm_us else [None] * 3
        eng._ar_dtop = fake("dtop", eng._ar_dtop, us3[1])
        eng._ar_drest = fake("drest", eng._ar_drest, us3[2])
        if schedule == "ddp":
            eng._ar_gparts = [fake("g[%d:%d]" % (lo, hi), r) for (_, lo, hi), r in zip(eng._g_cuts, eng._ar_gparts)]
        for name, r in list(vars(eng).items()):  # the G buckets of the segmented schedules
            if (name == "_ar_g" or name.startswith("_ar_gsplit")) and isinstance(r, D.GradAllReducer):
                setattr(eng, name, fake(name[4:], r, us3[0] if name == "_ar_g" else None))
    return eng, comm


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
    ap.add_argument("--fake_kind", default="rccl", choices=["rccl", "sleep"],
                    help="rccl: CU + HBM-consuming copy kernel (comm_emu.hip); sleep: round-3 timer")
    ap.add_argument("--fake_nwg", type=int, default=32, help="workgroups (RCCL channels) of the rccl stand-in")
    ap.add_argument("--allreduce_dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--graph", type=int, default=1, help="1: segment hipGraphs (rounds 2-5 numbers), 0: eager replay")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    ddp = a.schedule != "concurrent" or bool(a.fake_comm_us) or a.fake_busbw_gbs > 0
    eng, comm = standin_engine(cfg, a.batch_size, dev, schedule=a.schedule, ddp=ddp, graph=bool(a.graph),
                               wire=a.allreduce_dtype, busbw_gbs=a.fake_busbw_gbs, lat_us=a.fake_lat_us,
                               world=a.fake_world, kind=a.fake_kind, nwg=a.fake_nwg, comm_us=a.fake_comm_us,
                               timing=a.schedule in ("concurrent", "serial"))
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
    print(json.dumps({"schedule": eng._schedule(), "graph": eng.graph_enabled, "fake_kind": a.fake_kind,
                      "fake_world": a.fake_world, "fake_busbw_gbs": a.fake_busbw_gbs, "wire": a.allreduce_dtype,
                      "fake_comm_us": comm,
                      "ms_per_step_timed": round(ms, 4), "phases_ms": {k: round(v, 4) for k, v in acc.items()}}))


if __name__ == "__main__":
    main()
