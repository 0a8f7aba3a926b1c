"""Timing prototype of ONE D-backward data-gradient chain over 3B rows (round-6 review item 1).

Today's fused step runs two passes back through D: the d_loss chain over 2B rows [real | fake] on
alt0 (with D's weight gradients) and the g_loss chain over B fake rows on the main stream, ahead of
G's backward. The merged form runs one chain over 3B rows [real | fake.d_loss | fake.g_loss]:
one head backward, per layer one BN backward (3 statistics groups) and one data-gradient GEMM over
3B rows; D's weight gradients over the first 2B rows go to alt0 beside it (each after a mark on the
chain); D layer 0's image gradient runs over the g_loss rows only and feeds G's backward.

TIMING ONLY -- the numerics are not the step's: the activations of group 2 are separate rows
(random values written once; the real form would alias the fake rows, a kernel change this
prototype avoids), the head's dW / db, dgamma / dbeta and D layer 0's bias gradient also sum the
g_loss rows, and the head's BN statistics treat rows >= 2B as group 1. Kernel shapes, launch
counts, stream placement and bytes moved are the merged step's.

    python benchmarks/study/dmerge_proto.py --rounds 3 --steps 200 --warmup 20 [--tiles same2b]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_for_dcgan_amd.engine import hip_engine as HE  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig, same_pads  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.ops import hip as H  # noqa: E402

_p = HE._p
LRELU, TANH = HE.LRELU, HE.TANH


class MergedProto(HE.HipEngine):
    def _alloc(self):
        super()._alloc()
        B, t = self.B, self._t
        B2, B3 = 2 * B, 3 * B
        self.d_a3, self.d_x3 = {}, {}
        for L in self.dl:
            a3 = t(B3, L.out_hw, L.out_hw, L.cout)
            a3[B2:].copy_((torch.randn(a3[B2:].shape, device=self.device) * 0.5).to(a3.dtype))
            self.d_a3[L.name], self.d_a[L.name] = a3, a3[:B2]
            if L.bn:
                x3 = t(B3, L.out_hw, L.out_hw, L.cout)
                x3[B2:].copy_((torch.randn(x3[B2:].shape, device=self.device) * 0.5).to(x3.dtype))
                self.d_x3[L.name], self.d_x[L.name] = x3, x3[:B2]
        self.m_da = {L.name: t(B3, L.out_hw, L.out_hw, L.cout) for L in self.dl}
        self.m_dx = {L.name: t(B3, L.out_hw, L.out_hw, L.cout) for L in self.dl}
        self.dl3 = t(B3, dtype=torch.float32)
        self.dl_d, self.dl_g = self.dl3[:B2], self.dl3[B2:]
        for name, C in self.cfg.d_bn_layers():
            st = {k: t(3, C, dtype=torch.float32) for k in ("mean", "rstd", "scale", "shift")}
            st["mean"][2].zero_()
            st["rstd"][2].fill_(1.0)
            self.bn[name] = st
            self.coef[name] = t(3, C, 3, dtype=torch.float32)

    def _stats_buf(self, key, P, C):  # zeroed: the head never writes group 2's rows here
        buf = self._t(P, 2, C, dtype=torch.float32, zero=True)
        self._keep.append(buf)
        return buf

    def _build_d_backward_dloss(self, prog):
        self._b_split = 0  # progB stays empty: D's weight gradients are in progMW

    def _build_gloss_and_g_backward(self, prog, progw):
        cfg, B = self.cfg, self.B
        B2, B3 = 2 * B, 3 * B
        Pd, gD = self.model.d, self.grad_d
        lin = cfg.d_lin_name
        last = self.dl[-1]
        self.progMW, self._m_w = self._prog(), []
        # head backward over 3B rows (the kernel takes <= 2 statistics groups: rows >= 1.5B count as
        # group 1 here; group 2's partial rows stay zero -- timing only)
        C, K = last.cout, cfg.d_lin_in
        S = K // C
        part = self._stats_buf("m.d_head.bnstats", 3 * S, C)
        st = self.bn[last.bn]
        prog.head_bwd_rs("m.d_head.bwd", _p(self.d_a3[last.name]), _p(self.dl3), _p(Pd[lin + "/Matrix"]),
                         _p(self.m_da[last.name]), _p(gD[lin + "/Matrix"]), _p(gD[lin + "/bias"]), B3, K, 0,
                         _p(self.d_x3[last.name]), _p(self.d_a3[last.name]), _p(st["mean"]), _p(st["rstd"]), C,
                         B3 // 2, LRELU, cfg.lrelu_leak, _p(part), 1)
        fused_next = (part, S)
        for i in range(len(self.dl) - 1, -1, -1):
            L = self.dl[i]
            rows = B3 * L.out_hw ** 2
            da, a, dx = self.m_da[L.name], self.d_a3[L.name], self.m_dx[L.name]
            if L.bn:
                self._bn_bwd(prog, L.bn, self.d_x3[L.name], da, a, dx, rows, L.cout, 3, LRELU, Pd, gD,
                             self.coef[L.bn], write_param_grads=True, fused=fused_next)
            elif fused_next is not None:
                part, Pn = fused_next[0], fused_next[1]
                prog.sum_partials(L.name + ".dbias", _p(part), Pn, 2 * L.cout, L.cout, _p(gD[L.name + "/biases"]), 0)
            else:
                self._act_bwd_dbias(prog, L.name + ".act_bwd", da, a, dx, rows, L.cout, LRELU,
                                    gD[L.name + "/biases"], "d")
            # D's weight gradient over the d_loss rows, on alt0 once the chain has produced dx
            w0 = self.progMW.size()
            pad = same_pads(L.in_hw)[0]
            if i == 0:
                self.progMW.nwgrad(L.name + ".nwgrad", _p(self.d_in), B2, L.in_hw, L.in_hw, L.cin, _p(dx), L.out_hw,
                                   L.out_hw, pad, _p(gD[L.name + "/w"]), 0)
            else:
                src = self.d_a[self.dl[i - 1].name]
                self._wgrad(self.progMW, L.name, 0, src, L.in_hw, L.in_hw, L.cin, dx, B2, L.out_hw, L.out_hw,
                            L.cout, pad, gD[L.name + "/w"])
            self._m_w.append((prog.size(), self.progMW.size()))
            fused_next = None
            nat = self.wbf_d[L.name + "/w"]
            if i > 0:
                P_ = self.dl[i - 1]
                kw, out = {}, self.m_da[P_.name]
                if P_.bn:
                    r = self._dgrad_bnb(prog, 1, B3, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False,
                                        P_.bn, self.d_x3[P_.name], self.d_a3[P_.name], 3, LRELU)
                    if r is not None:
                        kw, fused_next = r[0], (r[1], r[2])
                else:
                    r = self._dgrad_actb(prog, 1, B3, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False,
                                         "m." + P_.name, self.d_a3[P_.name], LRELU)
                    if r is not None:
                        kw, fused_next, out = r[0], (r[1], r[2]), self.m_dx[P_.name]
                self._igemm(prog, "m." + L.name + ".dgrad", 1, dx, nat, out, B3, L.out_hw, L.out_hw, L.cout,
                            L.in_hw, L.in_hw, L.cin, pad, **kw)
            else:  # image gradient of the g_loss rows (+ G's tanh backward and output-bias gradient)
                assert self._img_dact()
                Lg = self.gl[-1]
                prog.narrow_deconv_dact("m." + L.name + ".dgrad_img+tanh_bwd", _p(dx[B2:]), _p(nat), _p(self.img_g),
                                        _p(self.fake), B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin,
                                        pad, TANH, 0.0, _p(self.grad_g[Lg.name + "/biases"]), 0)
        self._build_g_backward(prog, progw)

    def _run_fused(self, ex, cs):
        A = self.progA
        ex.run(A, [cs, ex.side], 0, self._a_fwd)
        a0, a1 = ex.alt
        ev = sorted([(ap, 0, k) for k, (ap, _) in enumerate(self._m_w)] +
                    [(ap, 1, k) for k, (ap, _) in enumerate(self._g_w)])
        pos = self._a_fwd
        for ap, kind, k in ev:
            ex.run(A, [cs, ex.side], pos, ap)
            pos = ap
            m = ex.mark(cs)
            if kind == 0:
                b = self._m_w[k - 1][1] if k > 0 else 0
                ex.wait_mark(a0, m)
                ex.run(self.progMW, [a0], b, self._m_w[k][1])
            else:
                b = self._g_w[k - 1][1] if k > 0 else 0
                ex.wait_mark(a1, m)
                ex.run(self.progW, [a1], b, self._g_w[k][1])
        ex.run(A, [cs, ex.side], pos, -1)
        ex.wait(cs, a0)
        ex.wait(cs, a1)
        ex.run(self.progC, [cs, ex.side])

    def kernel_count(self) -> int:
        return super().kernel_count() + sum(1 for i in range(self.progMW.size())
                                            if self.progMW.op_info(i)[2] == self.ext.OP_LAUNCH)


def _time(eng, steps, warmup):
    for _ in range(warmup):
        eng.train_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.train_step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--tiles", default="heur", help="heur | same2b (3B dgrads take the 2B dgrads' tuned tiles) | JSON")
    ap.add_argument("--check", action="store_true", help="schedule hazard check (dry run) and exit")
    a = ap.parse_args()
    cfg = DCGANConfig()
    B = 128
    if a.tiles != "heur":
        tab = H.tuned_table()
        if a.tiles == "same2b":
            for k, v in list(tab.items()):
                f = k.split(",")
                if f[0] == "1" and f[1] == str(2 * B):
                    tab[",".join([f[0], str(3 * B)] + f[2:])] = v
        else:
            for k, v in json.loads(a.tiles).items():
                c, sp = v.split(":")
                tab[k] = (int(c), int(sp))
    if a.check:
        from distributed_tensorflow_for_dcgan_amd.engine import schedule_check as SC
        eng = MergedProto(cfg, 8, torch.device("cpu"), dry_run=True, graph=False)
        hz, n = SC.check_engine(eng)
        print("merged proto: %d ops, %d hazards" % (n, len(hz)))
        for h in hz[:20]:
            print(" ", h)
        return
    dev = torch.device("cuda", 0)
    real = torch.rand(B, 64, 64, 3, device=dev) * 2 - 1
    e0 = HE.HipEngine(cfg, B, dev, graph=False)
    e1 = MergedProto(cfg, B, dev, graph=False)
    for e in (e0, e1):
        e.set_synthetic_batch(real)
    print("kernels/step: current %d, merged %d" % (e0.kernel_count(), e1.kernel_count()), flush=True)
    for r in range(a.rounds):
        t0 = _time(e0, a.steps, a.warmup)
        t1 = _time(e1, a.steps, a.warmup)
        print("round %d: current %.4f ms/step (%.0f img/s)  merged %.4f ms/step (%.0f img/s)  %+.2f %%"
              % (r, t0, B / t0 * 1e3, t1, B / t1 * 1e3, (t0 / t1 - 1) * 100), flush=True)


if __name__ == "__main__":
    main()
