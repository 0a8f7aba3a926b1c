"""Study: when do the two backward chains really start (no profiler)? The fused step's issue
sequence (HipEngine._run_fused) with GPU timing events after the forward, after the first few ops
of the G chain (main stream) and of the D chain (its own stream). rocprofv3 traces showed the G
chain's first kernel ~120 us after the forward (profiles/r5/step_profile_r5b.txt), but tracing
slows every launch on the host."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = HipEngine(DCGANConfig(), 128, dev, graph=False, seed=0)
    eng.set_batch(torch.rand(128, 64, 64, 3, device=dev) * 2 - 1)
    for _ in range(10):
        eng.train_step()
    ex = eng._get_exec()
    orig = eng._run_fused
    recs = []

    def timed(ex_, cs):
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("start", "fwd", "g1", "g3", "d1", "d3", "end")}
        ev["start"].record(cs)
        ex_.run(eng.progA, [cs, ex_.side], 0, eng._a_fwd)
        ev["fwd"].record(cs)
        ex_.wait(ex_.alt[0], cs)
        ex_.run(eng.progB, ex_.alt, 0, 1)
        ev["d1"].record(ex_.alt[0])
        ex_.run(eng.progB, ex_.alt, 1, 3)
        ev["d3"].record(ex_.alt[0])
        ex_.run(eng.progA, [cs, ex_.side], eng._a_fwd, eng._a_fwd + 1)
        ev["g1"].record(cs)
        ex_.run(eng.progA, [cs, ex_.side], eng._a_fwd + 1, eng._a_fwd + 3)
        ev["g3"].record(cs)
        # the rest exactly as _run_fused (its D chain re-runs progB[3:] etc.): finish the step
        ex_.run(eng.progB, ex_.alt, 3, -1)
        pos, marks = eng._a_fwd + 3, []
        for a_end, _ in eng._g_w:
            ex_.run(eng.progA, [cs, ex_.side], pos, a_end)
            marks.append(ex_.mark(cs))
            pos = a_end
        ex_.run(eng.progA, [cs, ex_.side], pos, -1)
        w, n_main = 0, min(eng._gw_tail_on_main(), len(eng._g_w))
        for m, (_, w_end) in zip(marks[:len(marks) - n_main], eng._g_w[:len(eng._g_w) - n_main]):
            ex_.wait_mark(ex_.alt[0], m)
            ex_.run(eng.progW, ex_.alt, w, w_end)
            w = w_end
        if n_main:
            ex_.run(eng.progW, [cs, ex_.side], w, -1)
        ex_.wait(cs, ex_.alt[0])
        ex_.run(eng.progC, [cs, ex_.side])
        ev["end"].record(cs)
        recs.append(ev)

    eng._run_fused = timed
    for _ in range(30):
        eng.train_step()
    torch.cuda.synchronize()
    eng._run_fused = orig
    rows = []
    for ev in recs[5:]:
        t = {k: ev["start"].elapsed_time(v) * 1e3 for k, v in ev.items() if k != "start"}
        rows.append(t)
    keys = ("fwd", "d1", "d3", "g1", "g3", "end")
    med = {k: sorted(r[k] for r in rows)[len(rows) // 2] for k in keys}
    print("median us from step start: " + "  ".join("%s %.1f" % (k, med[k]) for k in keys))
    print("G chain's first op ends %.1f us after the forward; the D chain's first op ends %.1f us after it"
          % (med["g1"] - med["fwd"], med["d1"] - med["fwd"]))


if __name__ == "__main__":
    main()
