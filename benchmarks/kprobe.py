#!/usr/bin/env python3
"""Run ONE conv-GEMM shape of the training step with given tile configs, a few times each --
a small, fixed workload for rocprofv3 PMC counter runs and A/B timing of kernel variants.

    python benchmarks/kprobe.py --shape D1.fwd --cfgs 210:1,100:1 [--reps 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_kernels import flops, shapes  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="D1.fwd")
    ap.add_argument("--cfgs", default="210:1")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--stamps", action="store_true", help="per-workgroup s_memtime phase breakdown (igemm3)")
    a = ap.parse_args()
    ext = H.ext()
    dev = torch.device("cuda", 0)
    sh = [s for s in shapes(DCGANConfig(output_size=64), a.batch) if s[0] == a.shape]
    if not sh:
        raise SystemExit("unknown shape %s" % a.shape)
    name, mode, Bn, Hin, Win, Kc, Hout, Wout, N, pad, bkn, kb = sh[0]
    if mode == 2:
        A = torch.randn(Bn * Hout * Wout, Kc, device=dev).to(torch.bfloat16)
    else:
        A = torch.randn(Bn, Hin, Win, Kc, device=dev).to(torch.bfloat16)
    Bw = (0.05 * torch.randn(25 * max(N, 8) * Kc, device=dev)).to(torch.bfloat16)
    C = torch.empty(Bn * Hout * Wout * N, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(1 << 22, device=dev)
    fl = flops(mode, Bn, Hin, Win, Kc, Hout, Wout, N)
    for spec in a.cfgs.split(","):
        c, sp = (int(x) for x in spec.split(":"))
        stamps = None
        if a.stamps:
            stamps = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
            os.environ["DCGAN_IGEMM_STAMPS"] = str(stamps.data_ptr())
        p = ext.Program()
        p.igemm_ex(name, mode, A.data_ptr(), Bw.data_ptr(), C.data_ptr(), Bn, Hin, Win, Kc, Hout, Wout, N, pad, pad,
                   c, 0, N, 0, 0, 0, 0.2, stats.data_ptr(), 0, bkn if c >= 200 else 0, kb if 200 <= c < 400 else -1, sp)
        H.run(p)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            H.run(p)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print("%s cfg %d:%d  %.1f us  %.0f TF/s" % (name, c, sp, us, fl / us / 1e6), flush=True)
        if stamps is not None:
            os.environ.pop("DCGAN_IGEMM_STAMPS", None)
            stamps.zero_()
            H.run(p)
            torch.cuda.synchronize()
            st = stamps.view(-1, 8).cpu()
            st = st[(st[:, 0] > 0) & (st[:, 3] > 0)].double()
            seg = {"decode": (0, 7), "prologue": (7, 1), "K loop": (1, 2), "split/sync": (2, 4),
                   "frag epilogue": (4, 5), "barrier": (5, 6), "stores+stats": (6, 3), "total": (0, 3)}
            print("  stamps (%d WGs, median cycles): " % st.shape[0] + ", ".join(
                "%s %d" % (k, (st[:, b] - st[:, a]).median()) for k, (a, b) in seg.items()), flush=True)


if __name__ == "__main__":
    main()
