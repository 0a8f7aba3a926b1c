"""In-situ tile tuning: pick each GEMM's (tile, LDS stages, split-K) by the WHOLE training step's
time instead of the kernel's isolated time (``bench_kernels.py`` / ``bench_wgrad.py``).

In the step, the D chain and the G chain run concurrently and every kernel shares the GPU with
another one, so the isolated optimum is not always the step optimum (a tile with fewer workgroups
can co-run better). Coordinate descent over the tuned-table entries the step uses: for each entry,
try its neighbours (half / double split-K, one more / one fewer LDS stage, a few sibling tiles),
rebuild the engine, time ``--steps`` graph-replayed steps, keep a change only if it beats the
incumbent by more than ``--min_gain``. One process, every candidate on the same GPU.

``--standin_world 8``: tune the segmented DDP step (what N = 2..8 ranks run) with the RCCL-like
stand-in collectives of ``benchmarks/phase_timing.py``; its table goes to ``--out`` only (a study:
``profiles/r5/ab_ddp_table_r5.txt``; the engine has one table for every schedule).

``python -m benchmarks.tune_insitu [--steps 150] [--passes 1] [--write]`` -- ``--write`` stores the
result in ops/igemm_tuned.json (the table the engine reads). Other image sizes / dtypes
(``--output_size 128``, ``--output_size 256 --batch 512 --dtype fp16``): the layers with no table
entry yet start from the heuristic's choice (``--seed``), so every GEMM of that step is tuned.
"""
import argparse
import gc
import json
import os
import time

import torch

from distributed_tensorflow_for_dcgan_amd.ops import hip as H
from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig


GRAPH = False  # --graph: time the hipGraph replay instead of the (default) C++ launch replay
STANDIN = None  # --standin_world W: time the segmented DDP step with RCCL-like stand-in collectives


def step_ms(cfg, B, steps, warmup, dtype="bf16"):
    dev = torch.device("cuda", 0)
    if STANDIN is not None:
        from benchmarks.phase_timing import standin_engine
        eng, _ = standin_engine(cfg, B, dev, graph=GRAPH, dtype=dtype, **STANDIN)
    else:
        eng = HipEngine(cfg, B, dev, seed=0, dtype=dtype, graph=GRAPH)
    real = torch.rand(B, cfg.output_size, cfg.output_size, cfg.c_dim, device=dev) * 2 - 1
    eng.set_synthetic_batch(real)
    for _ in range(warmup):
        eng.train_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.train_step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    del eng
    gc.collect()
    torch.cuda.empty_cache()
    return ms


def used_keys(cfg, B, dtype="bf16", seed=False):
    """Tuned-table keys the engine consults while building the step. seed=True: keys with no
    entry get the heuristic's (cfg, splits) as their entry (igemm3 / wgrad3 choices only)."""
    seen = []
    picked = {}
    orig_i, orig_w = H.igemm_cfg_for, H.wgrad3_cfg_for

    def log_i(mode, Bn, Hin, Win, Kc, Hout, Wout, N, *a, **k):
        key = "%d,%d,%d,%d,%d,%d,%d,%d" % (mode, Bn, Hin, Win, Kc, Hout, Wout, N)
        r = orig_i(mode, Bn, Hin, Win, Kc, Hout, Wout, N, *a, **k)
        if key not in seen:
            seen.append(key)
            picked[key] = r
        return r

    def log_w(Mc, Nc, Bn, Hd, Wd, Hg):
        key = H.wgrad3_key(Mc, Nc, Bn, Hd, Wd, Hg)
        r = orig_w(Mc, Nc, Bn, Hd, Wd, Hg)
        if key not in seen:
            seen.append(key)
            picked[key] = r
        return r

    H.igemm_cfg_for, H.wgrad3_cfg_for = log_i, log_w
    import distributed_tensorflow_for_dcgan_amd.engine.hip_engine as E
    E.H.igemm_cfg_for, E.H.wgrad3_cfg_for = log_i, log_w
    try:
        eng = HipEngine(cfg, B, torch.device("cuda", 0), seed=0, graph=False, dtype=dtype)
        del eng
    finally:
        H.igemm_cfg_for, H.wgrad3_cfg_for = orig_i, orig_w
        E.H.igemm_cfg_for, E.H.wgrad3_cfg_for = orig_i, orig_w
    gc.collect()
    torch.cuda.empty_cache()
    table = H.tuned_table()
    if seed:
        for k in seen:
            r = picked.get(k)
            if k not in table and r is not None and r[0] >= 200:
                table[k] = (int(r[0]), int(r[1]))
                print("  seed %-28s %d:%d (heuristic)" % (k, r[0], r[1]), flush=True)
    return [k for k in seen if k in table]


def neighbours(key, cur, tiles=False, extra_tiles=(), extra_cfgs=()):
    cfg, sp = cur
    out = []
    if not key.startswith("w3,"):  # explicit igemm3 configs (e.g. the ping-pong 24x / 25x), same split
        mode, Kc = int(key.split(",")[0]), int(key.split(",")[4])
        N = int(key.split(",")[7])
        out += [(c, sp) for c in extra_cfgs if H.igemm3_pp_ok(c, mode, Kc) and H.IGEMM3_TILES[c % 10][1] <= max(N, 64)]
    for s2 in (sp // 2, sp * 2, sp * 4, sp + 1, sp - 1):
        if 1 <= s2 <= 32 and s2 != sp:
            out.append((cfg, s2))
    if key.startswith("w3,"):
        f = key.split(",")  # w3,Mc,Nc,Bn,Hd,Wd,Hg
        Mc, Bn, Hd, Wd = int(f[1]), int(f[3]), int(f[4]), int(f[5])
        fam = [300, 301, 302, 303, 310, 311, 312, 313] + ([320, 322, 330, 332] if Mc == 64 else [])
        if not tiles:
            fam = {310: (311, 313), 311: (310, 313), 313: (311, 312), 312: (313, 311)}.get(cfg, ())
            if 300 <= cfg < 320:  # the same tile with the other LDS stage count (NS 3 <-> 2)
                fam = tuple(fam) + (cfg + 10 if cfg < 310 else cfg - 10,)
        # wgrad5 (halo rows) configurations that fit the layer
        fam = tuple(fam) + tuple(c for c in H.WGRAD5_CFGS if H.wgrad5_fits(c, Mc, Hd, Wd, Bn))
        out += [(c, sp) for c in fam]
    elif cfg >= 200:
        ns = (cfg - 200) // 10
        tile = cfg % 10
        for ns2 in (0, 1, 2):  # NS = 3 (20x), 2 (21x), 4 (22x)
            if ns2 != ns:
                out.append((200 + 10 * ns2 + tile, sp))
        for t2 in (range(9) if tiles else ()):
            if t2 != tile:
                out.append((200 + 10 * ns + t2, sp))
        for t2 in extra_tiles:  # e.g. --extra_tiles 9: the 8-wave 128x128 tile, same stages / split
            if t2 != tile:
                out.append((200 + 10 * ns + t2, sp))
    # igemm3 configs whose LDS ring does not fit 160 KiB are no candidates (e.g. 226: 8-wave 256x128 at NS = 4)
    out = [c for c in out if key.startswith("w3,") or c[0] < 200 or
           (c[0] % 10 in H.IGEMM3_TILES and H.igemm3_lds(c[0]) <= 160 * 1024 and H.igemm3_pp_ok(c[0], mode, Kc))]
    seen, res = set(), []
    for c in out:
        if c not in seen and c != cur:
            seen.add(c)
            res.append(c)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--passes", type=int, default=1)
    ap.add_argument("--min_gain", type=float, default=0.003, help="relative step-time gain to accept a change")
    ap.add_argument("--only", default="", help="comma-separated key prefixes")
    ap.add_argument("--keys", default="", help="'|'-separated full table keys")
    ap.add_argument("--tiles", action="store_true", help="also try sibling tiles (slower)")
    ap.add_argument("--extra_tiles", default="", help="comma-separated igemm3 tile ids to try on every GEMM entry")
    ap.add_argument("--extra_cfgs", default="", help="comma-separated igemm3 cfgs (e.g. 246,256) to try on every GEMM entry")
    ap.add_argument("--seed", action="store_true", help="tune layers with no table entry from the heuristic")
    ap.add_argument("--output_size", type=int, default=64)
    ap.add_argument("--c_dim", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--graph", type=int, default=0, help="1: tune under hipGraph replay (the pre-round-5 default)")
    ap.add_argument("--out", default="", help="also write the resulting table (JSON) here")
    ap.add_argument("--standin_world", type=int, default=0,
                    help="W > 0: tune the segmented DDP step (the N-GPU path) with the RCCL-like stand-in at W ranks")
    ap.add_argument("--standin_busbw", type=float, default=150.0, help="stand-in ring bus bandwidth (GB/s)")
    ap.add_argument("--standin_wire", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    global GRAPH, STANDIN
    GRAPH = bool(a.graph)
    if a.standin_world > 0:
        STANDIN = dict(world=a.standin_world, busbw_gbs=a.standin_busbw, wire=a.standin_wire)
    cfg = DCGANConfig(output_size=a.output_size, c_dim=a.c_dim)
    table = H.tuned_table()
    keys = used_keys(cfg, a.batch, a.dtype, a.seed)
    if a.only:
        keys = [k for k in keys if any(k.startswith(p) for p in a.only.split(","))]
    if a.keys:
        keys = [k for k in keys if k in a.keys.split("|")]
    print("keys in the step: %d" % len(keys), flush=True)
    best = step_ms(cfg, a.batch, a.steps, a.warmup, a.dtype)
    print("incumbent %.4f ms" % best, flush=True)
    log = []
    for ps in range(a.passes):
        for key in keys:
            cur = table[key]
            extra = tuple(int(x) for x in a.extra_tiles.split(",") if x)
            xcfg = tuple(int(x) for x in a.extra_cfgs.split(",") if x)
            for cand in neighbours(key, cur, a.tiles, extra, xcfg):
                table[key] = cand
                try:
                    ms = step_ms(cfg, a.batch, a.steps, a.warmup, a.dtype)
                except Exception as e:  # illegal combination for this layer: skip
                    print("  %s %d:%d failed: %s" % (key, cand[0], cand[1], str(e)[:80]), flush=True)
                    table[key] = cur
                    continue
                gain = (best - ms) / best
                print("  %-28s %d:%d -> %d:%d  %.4f ms (%+.2f%%)" % (key, cur[0], cur[1], cand[0], cand[1], ms,
                                                                     100 * gain), flush=True)
                log.append({"key": key, "from": "%d:%d" % cur, "to": "%d:%d" % cand, "ms": round(ms, 4)})
                if gain > a.min_gain:
                    cur, best = cand, ms
                    print("  * keep %s = %d:%d (%.4f ms)" % (key, cand[0], cand[1], ms), flush=True)
                else:
                    table[key] = cur
            table[key] = cur
        # re-measure the incumbent (noise guard for the next pass)
        best = step_ms(cfg, a.batch, a.steps, a.warmup, a.dtype)
        print("pass %d done: %.4f ms" % (ps + 1, best), flush=True)
    out = {k: "%d:%d" % v for k, v in sorted(table.items())}
    if a.out:
        json.dump({"table": out, "final_ms": best, "trials": log}, open(a.out, "w"), indent=1)
    if a.write:
        path = os.path.join(os.path.dirname(H.__file__), "igemm_tuned.json")
        json.dump(out, open(path, "w"), indent=1, sort_keys=True)
        print("wrote", path)


if __name__ == "__main__":
    main()
