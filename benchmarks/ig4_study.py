#!/usr/bin/env python3
"""igemm4 timing study: per layer shape, each cfg with the ablation bits of csrc/hip/igemm4.hip
(DCGAN_IGEMM_ABLATE: 1 = no fragment reads / MFMAs, 2 = no LDS-DMA, 3 = neither), next to the
best igemm3 tile -- interleaved rounds in one process (guide §5.4 rule 24).

    python benchmarks/ig4_study.py --only D1.fwd --cfgs 500,506 --ref 210:1
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_kernels import flops, shapes  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig, same_pads  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="D1.fwd")
    ap.add_argument("--cfgs", default="")
    ap.add_argument("--ref", default="")
    ap.add_argument("--ablate", default="0,1,2,3")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--inner", type=int, default=8)
    ap.add_argument("--stamps", action="store_true", help="per-workgroup s_memtime phases (igemm4 cfgs)")
    a = ap.parse_args()
    ext = H.ext()
    dev = torch.device("cuda", 0)
    for (name, mode, Bn, Hin, Win, Kc, Hout, Wout, N, pad, bkn, kb) in shapes(DCGANConfig(output_size=64), a.batch):
        if not any(o == name for o in a.only.split(",")):
            continue
        A = torch.randn(Bn, Hin, Win, Kc, device=dev).to(torch.bfloat16)
        Bw = (0.05 * torch.randn(25, N, Kc, device=dev)).to(torch.bfloat16)
        C = torch.empty(Bn * Hout * Wout * N, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(1 << 22, device=dev)
        fl = flops(mode, Bn, Hin, Win, Kc, Hout, Wout, N)
        cands = []
        if a.cfgs:
            for c in (int(x) for x in a.cfgs.split(",")):
                if H.igemm4_lds(c, mode, Bn, Kc, Hout, Wout, N, pad, pad) is not None and H.tile_of(c)[1] <= N:
                    for ab in (int(x) for x in a.ablate.split(",")):
                        cands.append((c, 1, ab))
        if a.ref:
            for spec in a.ref.split(","):
                c, sp = (int(x) for x in spec.split(":"))
                cands.append((c, sp, 0))
        progs = {}
        for (c, sp, ab) in cands:
            os.environ["DCGAN_IGEMM_ABLATE"] = str(ab)
            p = ext.Program()
            p.igemm_ex(name, mode, A.data_ptr(), Bw.data_ptr(), C.data_ptr(), Bn, Hin, Win, Kc, Hout, Wout, N, pad,
                       pad, c, 0, N, 0, 0, 0, 0.2, stats.data_ptr(), 0, bkn, kb if 200 <= c < 400 else -1, sp)
            progs[(c, sp, ab)] = p
        os.environ.pop("DCGAN_IGEMM_ABLATE", None)
        s = torch.cuda.current_stream()
        for c in cands:
            H.run(progs[c])
        torch.cuda.synchronize()
        times = {c: [] for c in cands}
        for _ in range(a.reps):
            for c in cands:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                H.run(progs[c])
                e0.record(s)
                for _ in range(a.inner):
                    H.run(progs[c])
                e1.record(s)
                times[c].append((e0, e1))
        torch.cuda.synchronize()
        if a.stamps:  # one extra launch per igemm4 cfg and ablation with stamps on
            for c in cands:
                if c[0] < 500:
                    continue
                st = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
                os.environ["DCGAN_IGEMM_STAMPS"] = str(st.data_ptr())
                os.environ["DCGAN_IGEMM_ABLATE"] = str(c[2])
                p = ext.Program()
                p.igemm_ex(name, mode, A.data_ptr(), Bw.data_ptr(), C.data_ptr(), Bn, Hin, Win, Kc, Hout, Wout, N, pad,
                           pad, c[0], 0, N, 0, 0, 0, 0.2, stats.data_ptr(), 0, bkn, -1, 1)
                os.environ.pop("DCGAN_IGEMM_STAMPS")
                os.environ.pop("DCGAN_IGEMM_ABLATE")
                H.run(p)
                torch.cuda.synchronize()
                nwg = p.last_mtiles() * (N // H.tile_of(c[0])[1])
                v = st[:nwg * 12].view(nwg, 12).cpu().double()
                t0 = v[:, 8].min()
                med = lambda x: float(x.median())  # noqa: E731
                print("%-12s cfg %d ablate %2d stamps (median cycles over %d WGs): entry->taps %.0f, taps->compute %.0f, "
                      "compute prologue->B0 %.0f, loop %.0f, "
                      "epilogue %.0f | loader issue-prologue %.0f, wait B0 %.0f, loop %.0f | WG span %.0f, "
                      "launch spread %.0f" % (name, c[0], c[2], nwg, med(v[:, 9] - v[:, 8]), med(v[:, 0] - v[:, 9]), med(v[:, 1] - v[:, 0]), med(v[:, 2] - v[:, 1]),
                                              med(v[:, 3] - v[:, 2]), med(v[:, 5] - v[:, 4]), med(v[:, 6] - v[:, 5]),
                                              med(v[:, 7] - v[:, 6]), med(v[:, 3] - v[:, 8]),
                                              float(v[:, 8].max() - t0)), flush=True)
        for c in cands:
            ts = sorted(e0.elapsed_time(e1) / a.inner for e0, e1 in times[c])
            med = ts[len(ts) // 2] * 1e3
            print("%-12s cfg %d:%d ablate %d  %7.1f us  %6.0f TF/s" % (name, c[0], c[1], c[2], med, fl / med / 1e6),
                  flush=True)


if __name__ == "__main__":
    main()
