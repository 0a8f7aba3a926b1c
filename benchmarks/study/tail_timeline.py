"""Study: what bounds the end of the fused 64x64 step (no profiler)? HipEngine._run_fused's issue
sequence with GPU timing events at the forward's end, the D chain's end, every G-chain mark (the
position where a G weight gradient's operand exists), the G chain's end, the end of every G
weight-gradient segment (D chain's stream or cs) and the end of Adam. Timing events cost a few us
each; the step end moves by that much against an untimed step.

    python benchmarks/study/tail_timeline.py [--tail-on-main N] [--place dscc]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tail-on-main", type=int, default=None)
    ap.add_argument("--place", default=None, help="DCGAN_GW_PLACE string (one of d/c/s/a per segment)")
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    if args.tail_on_main is not None:
        os.environ["DCGAN_GW_TAIL_ON_MAIN"] = str(args.tail_on_main)
    if args.place is not None:
        os.environ["DCGAN_GW_PLACE"] = args.place
    dev = torch.device("cuda", 0)
    eng = HipEngine(DCGANConfig(), 128, dev, graph=False, seed=0)
    eng.set_batch(torch.rand(128, 64, 64, 3, device=dev) * 2 - 1)
    for _ in range(10):
        eng.train_step()
    assert not eng._adam_early and eng._g_wgrad_on_d_stream()
    place = eng._gw_place()
    orig = eng._run_fused
    recs = []

    def timed(ex, cs):
        ev = {}

        def rec(k, s):
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            ev[k] = e

        rec("start", cs)
        ex.run(eng.progA, [cs, ex.side], 0, eng._a_fwd)
        rec("fwd", cs)
        ex.wait(ex.alt[0], cs)
        ex.run(eng.progB, ex.alt)
        rec("D_end", ex.alt[0])
        pos, marks = eng._a_fwd, []
        for j, (a_end, _) in enumerate(eng._g_w):
            ex.run(eng.progA, [cs, ex.side], pos, a_end)
            marks.append(ex.mark(cs))
            rec("G_mark%d" % j, cs)
            pos = a_end
        ex.run(eng.progA, [cs, ex.side], pos, -1)
        rec("G_end", cs)
        place = eng._gw_place()
        streams = {"d": ex.alt, "s": [ex.side], "a": [ex.alt[1]]}
        w, segs = 0, []
        for k, (m, (_, w_end)) in enumerate(zip(marks, eng._g_w)):
            segs.append((k, place[k], w, w_end))
            if place[k] != "c":
                st = streams[place[k]]
                ex.wait_mark(st[0], m)
                ex.run(eng.progW, st, w, w_end)
                rec("W%d_%s" % (k, place[k]), st[0])
            w = w_end
        for q in sorted(set(place) & {"s", "a"}):
            ex.wait(cs, streams[q][0])
        for k, q, lo, hi in segs:
            if q == "c":
                ex.run(eng.progW, [cs, ex.side], lo, hi)
                rec("W%d_c" % k, cs)
        ex.wait(cs, ex.alt[0])
        rec("join", cs)
        ex.run(eng.progC, [cs, ex.side], 0, -1)
        rec("end", cs)
        recs.append(ev)

    eng._run_fused = timed
    for _ in range(args.steps):
        eng.train_step()
    torch.cuda.synchronize()
    eng._run_fused = orig
    rows = [{k: ev["start"].elapsed_time(v) * 1e3 for k, v in ev.items() if k != "start"} for ev in recs[5:]]
    keys = list(rows[0])
    med = {k: sorted(r[k] for r in rows)[len(rows) // 2] for k in keys}
    print("placement %s (d: D chain's stream, c: cs after the G chain, s/a: side/alt1 stream)" % place)
    for k in sorted(keys, key=lambda k: med[k]):
        print("  %-10s %8.1f us" % (k, med[k]))


if __name__ == "__main__":
    main()
