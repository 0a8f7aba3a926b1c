"""Static stream-hazard checker for the HIP engine's training-step schedules.

The engine issues every schedule through an executor (``hip_engine._TorchExec``). This module
substitutes a recording executor and replays whole training steps of a *dry-run* engine -- its
``Program`` objects record ops, stream slots, cross-stream events and the exact device byte
ranges each op reads and writes (``csrc/bindings.cpp`` ``op_info``), without a GPU.

Each op gets a vector clock over the logical streams (main, side, alt0, alt1, comm): program
order on a stream, ``record``/``wait`` events inside programs, ``wait_stream``-style joins and
marks issued by the schedule, and the collectives on the comm stream. Two ops are *ordered*
when one's clock dominates the other's entry for its stream. Any unordered pair whose ranges
overlap with at least one write is a race (RAW / WAR / WAW) and is reported. Two consecutive
steps are recorded, so hazards across the step boundary are covered too.

Race this catches (round-1 finding): the timed single-process "concurrent" schedule ran the
one-launch two-model Adam in its "adam_G" segment, before the main stream had joined the D
chain -- Adam(D) read grad_d and rewrote D's weight mirror while D's backward still used them.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

STREAMS = ("main", "side", "alt0", "alt1", "comm")


@dataclass
class _Op:
    label: str
    stream: str
    vc: Dict[str, int]
    acc: List[Tuple[int, int, bool]]


@dataclass
class Hazard:
    a: str
    b: str
    kind: str
    addr: int
    nbytes: int

    def __str__(self) -> str:
        return "%s: %s  <->  %s  (0x%x, %d bytes)" % (self.kind, self.a, self.b, self.addr, self.nbytes)


class _S:
    def __init__(self, name: str):
        self.name = name

    def __repr__(self) -> str:
        return "<stream %s>" % self.name


class RecordingExec:
    """Drop-in for hip_engine._TorchExec that records instead of launching."""

    def __init__(self, ext):
        self.ext = ext
        st = {n: _S(n) for n in STREAMS}
        self._main = st["main"]
        self.side = st["side"]
        self.alt = [st["alt0"], st["alt1"]]
        self.comm = st["comm"]
        self.vc: Dict[str, Dict[str, int]] = {n: {n: 0} for n in STREAMS}
        self.ops: List[_Op] = []
        self.events: Dict[Tuple[int, int], Dict[str, int]] = {}
        self.step = 0

    def main(self):
        return self._main

    def _op(self, s: _S, label: str, acc) -> None:
        v = self.vc[s.name]
        v[s.name] = v.get(s.name, 0) + 1
        self.ops.append(_Op("step%d:%s" % (self.step, label), s.name, dict(v), list(acc)))

    @staticmethod
    def _merge(dst: Dict[str, int], src: Dict[str, int]) -> None:
        for k, x in src.items():
            if dst.get(k, 0) < x:
                dst[k] = x

    def run(self, prog, streams, begin: int = 0, end: int = -1) -> None:
        n = prog.size()
        end = n if end < 0 or end > n else end
        for i in range(begin, end):
            name, slot, kind, ev, acc = prog.op_info(i)
            if slot >= len(streams):
                raise RuntimeError("op %s uses stream slot %d of %d" % (name, slot, len(streams)))
            s = streams[slot]
            if kind == self.ext.OP_LAUNCH:
                self._op(s, name, acc)
            elif kind == self.ext.OP_RECORD:
                self.events[(id(prog), ev)] = dict(self.vc[s.name])
            else:
                key = (id(prog), ev)
                if key not in self.events:
                    raise RuntimeError("op %s waits on an event that was never recorded" % name)
                self._merge(self.vc[s.name], self.events[key])

    def wait(self, dst: _S, src: _S) -> None:
        self._merge(self.vc[dst.name], self.vc[src.name])

    def mark(self, stream: _S):
        return dict(self.vc[stream.name])

    def wait_mark(self, dst: _S, token) -> None:
        self._merge(self.vc[dst.name], token)

    def collective(self, reducer, stream: _S) -> None:
        label = getattr(reducer, "label", None) or "allreduce[%d elems]" % reducer.flat.numel()
        self._op(stream, label, reducer.accesses())

    def replay(self, graph, stream) -> None:  # graphs are never enabled in a dry run
        raise RuntimeError("graph replay in a recording executor")


def _ordered(a: _Op, b: _Op) -> bool:
    return a.vc[a.stream] <= b.vc.get(a.stream, 0) or b.vc[b.stream] <= a.vc.get(b.stream, 0)


def find_hazards(ops: List[_Op], limit: int = 50) -> List[Hazard]:
    """Unordered op pairs with overlapping byte ranges and at least one write (interval sweep)."""
    iv = []
    for k, op in enumerate(ops):
        for p, n, w in op.acc:
            if n > 0:
                iv.append((p, p + n, k, w))
    iv.sort()
    out: List[Hazard] = []
    seen = set()
    active: List[Tuple[int, int, int, bool]] = []
    for lo, hi, k, w in iv:
        active = [x for x in active if x[1] > lo]
        for lo2, hi2, k2, w2 in active:
            if k2 == k or not (w or w2):
                continue
            pair = (min(k, k2), max(k, k2))
            if pair in seen:
                continue
            a, b = ops[pair[0]], ops[pair[1]]
            if _ordered(a, b):
                continue
            seen.add(pair)
            kind = "WAW" if (w and w2) else "RAW/WAR"
            out.append(Hazard(a.label + "@" + a.stream, b.label + "@" + b.stream, kind, max(lo, lo2),
                              min(hi, hi2) - max(lo, lo2)))
            if len(out) >= limit:
                return out
        active.append((lo, hi, k, w))
    return out


def check_engine(eng, steps: int = 2) -> Tuple[List[Hazard], int]:
    """Record `steps` training steps of a dry-run HipEngine under its current schedule and
    return (hazards, ops recorded)."""
    if not eng.dry:
        raise ValueError("check_engine needs HipEngine(..., dry_run=True)")
    ex = RecordingExec(eng.ext)
    eng._ensure_comm()
    for s in range(steps):
        ex.step = s
        eng._run_step(ex)
    return find_hazards(ex.ops), len(ex.ops)


def check(cfg=None, batch_size: int = 8, dtype: str = "bf16", world: int = 1, schedule: Optional[str] = None,
          timing: bool = False, steps: int = 2, allreduce_dtype: str = "fp32"):
    """Build a dry-run engine on the CPU and check one schedule. Returns (schedule, hazards, ops)."""
    import torch

    from ..models.config import DCGANConfig
    from .hip_engine import HipEngine
    cfg = cfg or DCGANConfig()
    eng = HipEngine(cfg, batch_size, torch.device("cpu"), dtype=dtype, world=world, schedule=schedule, dry_run=True,
                    graph=False, allreduce_dtype=allreduce_dtype)
    if timing:  # (enable_timing without its CUDA events)
        eng._timing = True
        eng._build_updates()
    hz, n = check_engine(eng, steps)
    return eng._schedule(), hz, n


def main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description="stream-hazard check of every HIP engine schedule (CPU, dry run)")
    ap.add_argument("--batch_size", type=int, default=8)
    ap.add_argument("--output_size", type=int, default=64)
    args = ap.parse_args(argv)
    from ..models.config import DCGANConfig
    cfg = DCGANConfig(output_size=args.output_size)
    bad = 0
    for dtype in ("bf16", "fp16", "fp32"):
        for world, sched, timing in ((1, None, False), (1, None, True), (1, "serial", False), (2, None, False),
                                     (2, "ddp", False), (2, "serial", False)):
            s, hz, n = check(cfg, args.batch_size, dtype, world, sched, timing)
            print("%-5s W=%d %-10s timing=%d ops=%4d hazards=%d" % (dtype, world, s, timing, n, len(hz)))
            for h in hz[:10]:
                print("    ", h)
            bad += len(hz)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
