"""Time narrow2.hip (nconv / nwgrad) against the round-1 paths they replace, at the step's shapes
(64x64x3, B = 128 per half): D layer 0 forward (2B images), G's RGB-layer data gradient (B) and
both RGB weight gradients. ``python -m benchmarks.bench_narrow2 [--reps 50]``."""
import argparse
import json

import torch

from distributed_tensorflow_for_dcgan_amd.ops import hip as H


def timeit(prog, reps):
    H.run(prog)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        H.run(prog)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ext = H.ext()
    res = {}
    for name, B in (("D0.fwd(2B)", 2 * a.batch), ("G4.dgrad(B)", a.batch)):
        x = (torch.rand(B, 64, 64, 3, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(5, 5, 3, 64, device=dev) * 0.1).to(torch.bfloat16)
        bias = torch.rand(64, device=dev)
        y = torch.empty(B, 32, 32, 64, device=dev, dtype=torch.bfloat16)
        p_new = ext.Program()
        grid = H.nconv_grid(p_new, B, 32, 32)
        p_new.nconv("nc", H._p(x), H._p(w), H._p(bias), H._p(y), B, 64, 64, 3, 32, 32, 1, 1, 2, 0.2, grid,
                    0, 0, 0, 0, 0, 0.2, 0, 0)
        res[name] = {"nconv_us": timeit(p_new, a.reps)}
        if name.startswith("G4"):
            bx = torch.rand(B, 32, 32, 64, device=dev).to(torch.bfloat16)
            st = torch.rand(64, device=dev)
            part = torch.empty(grid, 2, 64, device=dev)
            p_b = ext.Program()
            p_b.nconv("ncb", H._p(x), H._p(w), 0, H._p(y), B, 64, 64, 3, 32, 32, 1, 1, 0, 0.2, grid,
                      H._p(bx), H._p(bx), H._p(st), H._p(st), 1, 0.2, H._p(part), 0)
            res[name]["nconv_bnb_us"] = timeit(p_b, a.reps)
            col = torch.empty(B * 32 * 32, 80, device=dev, dtype=torch.bfloat16)
            p_i = ext.Program()
            p_i.im2col_s2("i2c", H._p(x), H._p(col), B, 64, 64, 3, 32, 32, 1, 1, 80, 0)
            res[name]["im2col_us"] = timeit(p_i, a.reps)
    for name, B in (("D0.wgrad(2B)", 2 * a.batch), ("G4.wgrad(B)", a.batch)):
        x = (torch.rand(B, 64, 64, 3, device=dev) * 2 - 1).to(torch.bfloat16)
        d = (torch.rand(B, 32, 32, 64, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(25, 3, 64, device=dev)
        for cpw in (1, 2, 4, 8):
            p_c = ext.Program()
            p_c.nwgrad("nw", H._p(x), B, 64, 64, 3, H._p(d), 32, 32, 1, H._p(out), 0, cpw)
            res.setdefault(name, {})["nwgrad+reduce_cpw%d_us" % cpw] = timeit(p_c, a.reps)
        p_new = ext.Program()
        p_new.nwgrad("nw", H._p(x), B, 64, 64, 3, H._p(d), 32, 32, 1, H._p(out), 0)
        col = torch.empty(B * 32 * 32, 80, device=dev, dtype=torch.bfloat16)
        cfg, splits = H.pick_wgrad(80, 64, B * 1024, 1, dtype=0)
        slabs = torch.empty(splits, 1, 80, 64, device=dev)
        p_old = ext.Program()
        p_old.im2col_s2("i2c", H._p(x), H._p(col), B, 64, 64, 3, 32, 32, 1, 1, 80, 0)
        p_old.wgrad("wg", 2, H._p(col), 1, 1, 80, H._p(d), B * 1024, 1, 1, 64, 0, cfg, splits, H._p(slabs),
                    H._p(out), 75 * 64, 1.0, 0)
        res[name].update({"im2col+wgrad+reduce_us": timeit(p_old, a.reps), "nwgrad+reduce_us": timeit(p_new, a.reps)})
    for k, v in res.items():
        print(json.dumps({"shape": k, **{kk: round(vv, 2) for kk, vv in v.items()}}))


if __name__ == "__main__":
    main()
