#!/usr/bin/env python3
"""Per-layer kernel benchmark / autotuner for the implicit-GEMM conv kernel (MI355X).

For every conv-shaped GEMM of the DCGAN training step (D forward on 2B, D dgrads, G forward,
G dgrads, at per-GPU batch B) time every tile configuration and both staging variants
(register staging vs LDS-DMA) in ONE process, interleaved (guide §5.4 rule 24), and report
TF/s. ``--write`` stores the fastest config per shape in ops/igemm_tuned.json, which the
engine's tile policy consults first.

    python benchmarks/bench_kernels.py --batch 128 [--write] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig, same_pads  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.ops import hip as H  # noqa: E402


def shapes(cfg: DCGANConfig, B: int):
    """(name, mode, Bn, Hin, Win, Kc, Hout, Wout, N, pad, flops)"""
    out = []
    for i, L in enumerate(cfg.d_layers()):
        pad = same_pads(L.in_hw)[0]
        if L.cin % 8 == 0:
            out.append(("D%d.fwd" % i, 0, 2 * B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad))
        else:
            out.append(("D%d.fwd(im2col)" % i, 2, 2 * B, 1, 1, -(-25 * L.cin // 16) * 16, L.out_hw, L.out_hw, L.cout, 0))
        if i > 0:
            out.append(("D%d.dgrad2B" % i, 1, 2 * B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad))
        out.append(("D%d.dgradB" % i, 1, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad))
    for L in cfg.g_layers():
        pad = same_pads(L.out_hw)[0]
        out.append(("G.%s.fwd" % L.name, 1, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad))
        if L.cout % 8 == 0:
            out.append(("G.%s.dgrad" % L.name, 0, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad))
        else:
            out.append(("G.%s.dgrad(im2col)" % L.name, 2, B, 1, 1, -(-25 * L.cout // 16) * 16, L.in_hw, L.in_hw,
                        L.cin, 0))
    return out


def flops(mode, Bn, Hin, Win, Kc, Hout, Wout, N):
    if mode == 0:
        return 2.0 * Bn * Hout * Wout * N * Kc * 25
    if mode == 1:
        return 2.0 * Bn * Hout * Wout * N * Kc * 25 / 4
    return 2.0 * Bn * Hout * Wout * N * Kc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    cfg = DCGANConfig(output_size=a.size)
    ext = H.ext()
    dev = torch.device("cuda", 0)
    table = {}
    for (name, mode, Bn, Hin, Win, Kc, Hout, Wout, N, pad) in shapes(cfg, a.batch):
        if a.only and a.only not in name:
            continue
        if mode == 2:
            A = torch.randn(Bn * Hout * Wout, Kc, device=dev).to(torch.bfloat16)
            Bw = torch.randn(N, Kc, device=dev).to(torch.bfloat16)
        else:
            A = torch.randn(Bn, Hin, Win, Kc, device=dev).to(torch.bfloat16)
            Bw = (0.05 * torch.randn(25, N, Kc, device=dev)).to(torch.bfloat16)
        C = torch.empty(Bn * Hout * Wout * N, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(1 << 22, device=dev)
        fl = flops(mode, Bn, Hin, Win, Kc, Hout, Wout, N)
        cands = []
        for c, (bm, bn) in H.IGEMM_CFGS.items():
            if (N <= 16) != (bn == 16):
                continue
            if bn > 32 and N < bn:
                continue
            for st in (0, 100):
                cands.append(c + st)
        progs = {}
        for c in cands:
            p = ext.Program()
            p.igemm(name, mode, A.data_ptr(), Bw.data_ptr(), C.data_ptr(), Bn, Hin, Win, Kc, Hout, Wout, N, pad, pad,
                    c, 0, N, 0, 0, 0, 0.2, stats.data_ptr(), 0)
            progs[c] = p
        times = {c: [] for c in cands}
        s = torch.cuda.current_stream()
        for c in cands:  # warm
            H.run(progs[c])
        torch.cuda.synchronize()
        for _ in range(a.reps):
            for c in cands:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                H.run(progs[c])
                e1.record(s)
                times[c].append((e0, e1))
        torch.cuda.synchronize()
        res = []
        for c in cands:
            ts = sorted(e0.elapsed_time(e1) for e0, e1 in times[c])
            med = ts[len(ts) // 2] * 1e3
            res.append((med, c))
        res.sort()
        best = res[0]
        print("%-22s M/ph=%7d N=%4d K=%5d  best cfg %3d %-10s %7.1f us %6.0f TF/s | " %
              (name, Bn * Hout * Wout // (4 if mode == 1 else 1), N, Kc * (25 if mode == 0 else 1), best[1],
               H.IGEMM_CFGS[best[1] % 100], best[0], fl / best[0] / 1e6) +
              " ".join("%d:%.0f" % (c, t) for t, c in res[:6]), flush=True)
        table["%d,%d,%d,%d,%d,%d,%d,%d" % (mode, Bn, Hin, Win, Kc, Hout, Wout, N)] = best[1]
    if a.write:
        path = os.path.join(os.path.dirname(H.__file__), "igemm_tuned.json")
        old = {}
        if os.path.exists(path):
            old = json.load(open(path))
        old.update(table)
        json.dump(old, open(path, "w"), indent=1, sort_keys=True)
        print("wrote", path)


if __name__ == "__main__":
    main()
