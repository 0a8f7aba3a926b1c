#!/usr/bin/env python3
"""Weight-gradient kernel benchmark / autotuner (MI355X).

For every 25-tap weight gradient of the DCGAN training step (D layers on the 2B batch, G layers
on B) time the register-staged wgrad.hip kernel (+ its split-K reduce pass) and every
wgrad3.hip configuration (tile x LDS stages x split-K, reduction in-kernel) in ONE process,
interleaved (guide §5.4 rule 24), check each result against wgrad.hip's, and report TF/s.
``--write`` stores the fastest as "cfg:splits" under key "w3,Mc,Nc,Bn,Hd,Wd,Hg" in
ops/igemm_tuned.json (cfg 0 = keep wgrad.hip); the engine's tile policy consults it first.

    python benchmarks/bench_wgrad.py --batch 128 [--size 64] [--write]
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
    """(name, Bn, Hg, Wg, Mc, Hd, Wd, Nc, pad) exactly as HipEngine._wgrad is called: G = the
    gathered operand (layer input for D, dL/d(out) for G), Dm = the direct one."""
    out = []
    for i, L in enumerate(cfg.d_layers()):
        if L.cin % 8 == 0:
            out.append(("D%d.wgrad" % i, 2 * B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout,
                        same_pads(L.in_hw)[0]))
    for L in cfg.g_layers():
        if L.cout % 8 == 0:
            out.append(("G.%s.wgrad" % L.name, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin,
                        same_pads(L.out_hw)[0]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--write", action="store_true")
    a = ap.parse_args()
    cfg = DCGANConfig(output_size=a.size)
    ext = H.ext()
    dev = torch.device("cuda", 0)
    table = {}
    for (name, Bn, Hg, Wg, Mc, Hd, Wd, Nc, pad) in shapes(cfg, a.batch):
        G = torch.randn(Bn, Hg, Wg, Mc, device=dev).to(torch.bfloat16)
        Dm = torch.randn(Bn, Hd, Wd, Nc, device=dev).to(torch.bfloat16)
        K = Bn * Hd * Wd
        fl = 2.0 * 25 * Mc * Nc * K
        kt = -(-K // 64)
        progs, outs = {}, {}
        c0, s0 = H.pick_wgrad(Mc, Nc, K, 25)
        keep = []
        for sw in sorted({s0, 4, 8, 12, 16, 24, 32}):  # wgrad.hip (+ its slab reduce) at several split counts
            if sw > 1 and kt // sw < 4:
                continue
            slabs = torch.empty(sw, 25, Mc, Nc, device=dev)
            keep.append(slabs)
            outs[(0, sw)] = torch.empty(25, Mc, Nc, device=dev)
            p = ext.Program()
            p.wgrad(name, 0, G.data_ptr(), Hg, Wg, Mc, Dm.data_ptr(), Bn, Hd, Wd, Nc, pad, c0, sw, slabs.data_ptr(),
                    outs[(0, sw)].data_ptr(), 25 * Mc * Nc, 1.0, 0)
            progs[(0, sw)] = p
        for c3 in (300, 301, 302, 303, 310, 311, 312, 313, 320, 322, 330, 332):
            bm, bn = H.WGRAD3_TILES[c3 % 10]
            if c3 >= 320:  # two taps per tile: BM = 2 Mc
                if 2 * Mc != bm or bn > max(Nc, 64):
                    continue
            elif bm > max(Mc, 64) or bn > max(Nc, 64):
                continue
            for sp in (1, 2, 4, 8, 16, 24, 32):
                if sp > 1 and kt // sp < 4:
                    continue
                o = torch.empty(25, Mc, Nc, device=dev)
                p = ext.Program()
                p.wgrad3(name, G.data_ptr(), Hg, Wg, Mc, Dm.data_ptr(), Bn, Hd, Wd, Nc, pad, c3, sp, o.data_ptr(), 1.0, 0)
                progs[(c3, sp)], outs[(c3, sp)] = p, o
        for c5 in sorted(H.WGRAD5_CFGS):  # wgrad5.hip: halo rows, one kernel row of taps per workgroup
            if not H.wgrad5_fits(c5, Mc, Hd, Wd, Bn):
                continue
            for sp in (1, 2, 4, 8, 16, 24, 32, 48, 64):
                if sp > 1 and kt // sp < 4:
                    continue
                o = torch.empty(25, Mc, Nc, device=dev)
                p = ext.Program()
                p.wgrad3(name, G.data_ptr(), Hg, Wg, Mc, Dm.data_ptr(), Bn, Hd, Wd, Nc, pad, c5, sp, o.data_ptr(), 1.0, 0)
                progs[(c5, sp)], outs[(c5, sp)] = p, o
        cands = list(progs)
        s = torch.cuda.current_stream()
        for c in cands:
            H.run(progs[c])
        torch.cuda.synchronize()
        ref = outs[(0, s0)]
        scale = ref.abs().max().item()
        bad = {c for c in cands if (outs[c] - ref).abs().max().item() > 1e-3 * scale}
        times = {c: [] for c in cands}
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
            res.append((ts[len(ts) // 2] * 1e3, c))
        res.sort()
        good = [r for r in res if r[1] not in bad]
        best_t, (bc, bsp) = good[0]
        old_t = [t for t, c in res if c == (0, s0)][0]
        print("%-14s Mc=%4d Nc=%4d K=%7d  wgrad.hip %7.1f us | best %3d:%-2d %7.1f us %6.0f TF/s | bad %s | %s" %
              (name, Mc, Nc, K, old_t, bc, bsp, best_t, fl / best_t / 1e6, sorted(bad) or "-",
               " ".join("%d:%d:%.0f" % (c[0], c[1], t) for t, c in good[:6])), flush=True)
        w5 = [r for r in good if r[1][0] >= 400]
        if w5:
            print("%-14s   wgrad5: %s" % (name, " ".join("%d:%d:%.1f" % (c[0], c[1], t) for t, c in w5[:8])), flush=True)
        table[H.wgrad3_key(Mc, Nc, Bn, Hd, Wd, Hg)] = "%d:%d" % (bc, bsp)
    if a.write:
        path = H.TUNED_PATH
        old = json.load(open(path)) if os.path.exists(path) else {}
        old.update(table)
        json.dump(old, open(path, "w"), indent=1, sort_keys=True)
        print("wrote", path)


if __name__ == "__main__":
    main()
