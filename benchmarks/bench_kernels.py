#!/usr/bin/env python3
"""Per-layer kernel benchmark / autotuner for the implicit-GEMM conv kernel (MI355X).

For every conv-shaped GEMM of the DCGAN training step (D forward on 2B, D dgrads, G forward,
G dgrads, at per-GPU batch B) time every tile configuration -- igemm.hip (both staging
variants) and igemm3.hip (every tile, 2..5 LDS stages, split-K 1..8) with the weight layout
the engine reads for that GEMM -- in ONE process, interleaved (guide §5.4 rule 24), and
report TF/s. ``--write`` stores the fastest "cfg:splits" per shape in ops/igemm_tuned.json,
which the engine's tile policy consults first.

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
    """(name, mode, Bn, Hin, Win, Kc, Hout, Wout, N, pad, bkn, kb_valid). bkn = weight layout the
    engine reads: the TF layout itself, which is [tap][K][N] for D forward / G dgrad and
    [tap][N][K] for D dgrad / G forward."""
    out = []
    for i, L in enumerate(cfg.d_layers()):
        pad = same_pads(L.in_hw)[0]
        if L.cin % 8 == 0:
            out.append(("D%d.fwd" % i, 0, 2 * B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad, 1, -1))
        else:
            out.append(("D%d.fwd(im2col)" % i, 2, 2 * B, 1, 1, -(-25 * L.cin // 16) * 16, L.out_hw, L.out_hw, L.cout,
                        0, 1, 25 * L.cin))
        if i > 0:
            out.append(("D%d.dgrad2B" % i, 1, 2 * B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad, 0, -1))
        out.append(("D%d.dgradB" % i, 1, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad, 0, -1))
    for L in cfg.g_layers():
        pad = same_pads(L.out_hw)[0]
        out.append(("G.%s.fwd" % L.name, 1, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad, 0, -1))
        if L.cout % 8 == 0:
            out.append(("G.%s.dgrad" % L.name, 0, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad, 1, -1))
        else:
            out.append(("G.%s.dgrad(im2col)" % L.name, 2, B, 1, 1, -(-25 * L.cout // 16) * 16, L.in_hw, L.in_hw,
                        L.cin, 0, 1, 25 * L.cout))
    return out


V1 = False  # --v1: also time the first-generation igemm.hip tiles


def candidates(mode, Bn, Hout, Wout, Kc, N, bkn):
    """[(cfg, splits)] worth timing for one GEMM."""
    out = []
    if not bkn and V1:  # igemm.hip reads k-contiguous weights only
        for c, (bm, bn) in H.IGEMM_CFGS.items():
            if (N <= 16) != (bn == 16):
                continue
            if bn > 32 and N < bn:
                continue
            out += [(c, 1), (c + 100, 1)]
    if N % 8 or N <= 16:
        return out
    phases = 4 if mode == 1 else 1
    M = Bn * (-(-Hout // 2)) * (-(-Wout // 2)) if mode == 1 else Bn * Hout * Wout
    kt = (9 if mode == 1 else 25 if mode == 0 else 1) * -(-Kc // 64)
    for c in range(200, 260):
        if c % 10 not in H.IGEMM3_TILES or H.igemm3_lds(c) > 160 * 1024:
            continue
        if not H.igemm3_pp_ok(c, mode, Kc):
            continue
        bm, bn = H.IGEMM3_TILES[c % 10]
        if bn > N:
            continue
        tiles = -(-M // bm) * -(-N // bn) * phases
        for sp in (1, 2, 3, 4, 6, 8):
            if sp > 1 and (kt // sp < 2 or tiles * sp > 4096):
                continue
            if sp > 1 and tiles >= 1024:
                continue
            out.append((c, sp))
    if mode == 1 and not bkn:  # the halo K loop (deconv phases): split-K over 64-channel chunks
        for c in range(300, 320):
            for sp in (1, 2, 4):
                if H.halo_ok(c, mode, Bn, Hout, Wout, Kc, False, sp):
                    out.append((c, sp))
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
    ap.add_argument("--inner", type=int, default=8, help="launches per timed event pair")
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--v1", action="store_true", help="also time igemm.hip (v1) tiles")
    ap.add_argument("--out", default="", help="also write this run's table (JSON) here")
    ap.add_argument("--top", type=int, default=6, help="candidates listed per shape")
    ap.add_argument("--cfgs", default="", help="comma-separated cfg prefix filter, e.g. 4,21")
    a = ap.parse_args()
    global V1
    V1 = a.v1
    cfg = DCGANConfig(output_size=a.size)
    ext = H.ext()
    dev = torch.device("cuda", 0)
    table = {}
    for (name, mode, Bn, Hin, Win, Kc, Hout, Wout, N, pad, bkn, kb) in shapes(cfg, a.batch):
        if a.only and a.only not in name:
            continue
        if mode == 2:
            A = torch.randn(Bn * Hout * Wout, Kc, device=dev).to(torch.bfloat16)
            Bw = torch.randn(max(N, 8) * Kc, device=dev).to(torch.bfloat16)
        else:
            A = torch.randn(Bn, Hin, Win, Kc, device=dev).to(torch.bfloat16)
            Bw = (0.05 * torch.randn(25, N, Kc, device=dev)).to(torch.bfloat16)
        C = torch.empty(Bn * Hout * Wout * N, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(1 << 22, device=dev)
        fl = flops(mode, Bn, Hin, Win, Kc, Hout, Wout, N)
        cands = candidates(mode, Bn, Hout, Wout, Kc, N, bkn)
        if a.cfgs:
            cands = [c for c in cands if any(str(c[0]).startswith(f) for f in a.cfgs.split(","))]
        if not cands:
            print("%-22s (no igemm3 tile: N=%d)" % (name, N))
            continue
        progs = {}
        for (c, sp) in cands:
            p = ext.Program()
            p.igemm_ex(name, mode, A.data_ptr(), Bw.data_ptr(), C.data_ptr(), Bn, Hin, Win, Kc, Hout, Wout, N, pad,
                       pad, c, 0, N, 0, 0, 0, 0.2, stats.data_ptr(), 0, bkn if c >= 200 else 0,
                       kb if 200 <= c < 400 else -1, sp)  # noqa
            progs[(c, sp)] = p
        times = {c: [] for c in cands}
        s = torch.cuda.current_stream()
        for c in cands:  # warm
            H.run(progs[c])
        torch.cuda.synchronize()
        for _ in range(a.reps):
            for c in cands:
                # `inner` back-to-back launches per event pair: the host launch latency of the
                # first one is not counted against the kernel (the queue stays full after it)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                H.run(progs[c])
                e0.record(s)
                for _ in range(a.inner):
                    H.run(progs[c])
                e1.record(s)
                times[c].append((e0, e1))
        torch.cuda.synchronize()
        res = []
        for c in cands:
            ts = sorted(e0.elapsed_time(e1) / a.inner for e0, e1 in times[c])
            med = ts[len(ts) // 2] * 1e3
            res.append((med, c))
        res.sort()
        best = res[0]
        bc, bsp = best[1]
        print("%-22s M/ph=%7d N=%4d K=%5d  best %3d:%d %-10s %7.1f us %6.0f TF/s | " %
              (name, Bn * Hout * Wout // (4 if mode == 1 else 1), N, Kc * (25 if mode == 0 else 1), bc, bsp,
               H.tile_of(bc), best[0], fl / best[0] / 1e6) +
              " ".join("%d:%d:%.0f" % (c[0], c[1], t) for t, c in res[:a.top]), flush=True)
        table["%d,%d,%d,%d,%d,%d,%d,%d" % (mode, Bn, Hin, Win, Kc, Hout, Wout, N)] = "%d:%d" % (bc, bsp)
    if a.out:
        json.dump(table, open(a.out, "w"), indent=1, sort_keys=True)
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
