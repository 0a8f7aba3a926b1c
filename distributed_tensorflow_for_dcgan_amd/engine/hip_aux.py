"""Observability / inference helpers of the HIP engine (mixin of ``hip_engine.HipEngine``): views
of the last step's tensors, on-device TensorBoard summaries, the EMA-BN sampler
(``distriubted_model.py:131-153``), sample-time losses (``image_train.py:181-184``) and the
launch / placement accounting behind ``--log_device_placement`` and bench.py's kernel count. None
of it runs inside the training step."""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List

import torch

from ..models.config import same_pads
from ..ops import hip as H

RELU, TANH = 1, 3


def _p(t) -> int:
    return 0 if t is None else int(t.data_ptr())


class HipEngineAux:
    def activations(self) -> "Dict[str, torch.Tensor]":
        """Views of the last step's tensors for summaries (no extra compute)."""
        B = self.B
        a = OrderedDict()
        a["z"] = self.z
        a["d"] = self.prob[:B]
        a["d_"] = self.prob[B:]
        a["G"] = self.fake
        a["g_h0_relu"] = self.g_h0
        for L in self.gl[:-1]:
            a[L.name + "_relu"] = self.g_a[L.name]
        a[self.gl[-1].name] = self.fake
        for L in self.dl:
            a[L.name] = self.d_a[L.name][:B]
        a[self.cfg.d_lin_name] = self.logits[:B]
        return a

    # ------------------------------------------------------------------ device-side summaries
    def device_summaries(self) -> "OrderedDict[str, object]":
        """Zero fraction + TF-bucket histogram statistics of every summarised tensor, computed on
        the device (summary.hip) in ONE program; only the per-tensor statistics rows (a few KB
        each) are copied to the host. Returns name -> numpy row [min, max, n, sum, sumsq, zeros,
        counts...] (obs.summaries turns them into TensorBoard protos)."""
        from ..obs.events import BUCKET_EDGES
        if self.progSum is None:
            names, tensors = [], []
            for name, t in self.activations().items():
                if name != "G":
                    names.append(name + ("/activations" if name not in ("z", "d", "d_") else ""))
                    tensors.append(t)
            sharded = getattr(self, "_shards", None) is not None and self._sharded()
            for name, t in self.model.all_named_variables().items():
                if sharded and name.endswith("/w"):  # masters current only on this rank's shard:
                    mir = self.wbf_g if name in self.wbf_g.tensors else self.wbf_d  # the bf16 mirror
                    t = mir[name]
                names.append(name)
                tensors.append(t)
            nb = len(BUCKET_EDGES) + 1
            self._sum_edges = torch.tensor(BUCKET_EDGES, dtype=torch.float64, device=self.device)
            self._sum_out = torch.zeros(len(tensors), nb + 6, dtype=torch.float64, device=self.device)
            prog = self._prog()
            for i, t in enumerate(tensors):
                xd = 0 if t.dtype == torch.float32 else 1
                if xd == 1 and t.dtype != self.edt:
                    raise TypeError("summary of %s: dtype %s" % (names[i], t.dtype))
                prog.tensor_summary("sum." + names[i], _p(t), xd, t.numel(), _p(self._sum_edges), nb,
                                    _p(self._sum_out[i]), 0)
            self.progSum, self._sum_names = prog, names
        H.run(self.progSum)
        rows = self._sum_out.cpu().numpy()
        return OrderedDict(zip(self._sum_names, rows))

    # ------------------------------------------------------------------ sampling / eval
    def sampler(self, z: torch.Tensor) -> torch.Tensor:
        """G with inference-mode BN (moving averages) -- distriubted_model.py:131-153. With
        --bn_zero_debias the moving averages are divided by 1 - decay^t (t = EMA updates so far,
        as in the reference engine's BNState.averages)."""
        if self.progS is None:
            self._build_sampler()
        bn = self.model.g_bn
        t = float(bn.steps[0])
        corr = 1.0 - bn.decay ** t if (bn.zero_debias and t > 0) else 1.0
        self._debias.fill_(1.0 / corr)
        self.sample_z.copy_(z.to(self.device, torch.float32))
        H.run(self.progS)
        return self._s_out.float().clone()

    def _build_sampler(self):
        cfg, B = self.cfg, self.B
        prog = self._prog()
        Pg = self.model.g
        t = self._t
        h0p, h0 = t(B, cfg.g_lin_out), t(B, cfg.g_lin_out)
        self._s_out = t(B, cfg.output_size, cfg.output_size, cfg.c_dim)
        sc = {name: (t(C, dtype=torch.float32), t(C, dtype=torch.float32)) for name, C in cfg.g_bn_layers()}
        self._s_keep = [h0p, h0, sc]
        bnst = self.model.g_bn
        prog.linear_fwd("s.lin", _p(self.sample_z), _p(Pg["g_h0_lin/Matrix"]), _p(Pg["g_h0_lin/bias"]), _p(h0p), B,
                        cfg.z_dim, cfg.g_lin_out, 0)

        def coef(name, C):  # BN state and the debias factor are read live (device pointers)
            prog.bn_coef_eval("s." + name, C, _p(Pg[name + "/gamma"]), _p(Pg[name + "/beta"]), cfg.bn_eps,
                              _p(bnst.mean[name]), _p(bnst.var[name]), 1.0, _p(sc[name][0]), _p(sc[name][1]), 0,
                              _p(self._debias))

        C0 = cfg.g_base_ch
        coef("g_bn0", C0)
        prog.bn_apply_act("s.g_bn0", _p(h0p), _p(h0), _p(sc["g_bn0"][0]), _p(sc["g_bn0"][1]),
                          B * cfg.g_base_hw ** 2, C0, B * cfg.g_base_hw ** 2, RELU, 0.0, 0)
        prev = h0
        for L in self.gl:
            nat = self.wbf_g[L.name + "/w"]
            pad = same_pads(L.out_hw)[0]
            if L.bn:
                xb, ab = t(B, L.out_hw, L.out_hw, L.cout), t(B, L.out_hw, L.out_hw, L.cout)
                self._s_keep += [xb, ab]
                self._igemm(prog, "s." + L.name, 1, prev, nat, xb, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw,
                            L.cout, pad, bias=Pg[L.name + "/biases"])
                coef(L.bn, L.cout)
                rows = B * L.out_hw ** 2
                prog.bn_apply_act("s." + L.bn, _p(xb), _p(ab), _p(sc[L.bn][0]), _p(sc[L.bn][1]), rows, L.cout, rows,
                                  RELU, 0.0, 0)
                prev = ab
            else:
                self._deconv_out(prog, "s." + L.name, prev, nat, self._s_out, B, L, pad, Pg[L.name + "/biases"], TANH)
        self.progS = prog

    def eval_losses(self, real: torch.Tensor, z: torch.Tensor) -> Dict[str, float]:
        """Sample-time d_loss / g_loss (image_train.py:181-184) in train-mode BN but WITHOUT
        mutating the moving averages (documented deviation)."""
        if self.progEval is None:
            prog = self._prog()
            self._ev_z = self._t(self.B, self.cfg.z_dim, dtype=torch.float32)
            self._build_forward(prog, update_ema=False, z=self._ev_z, train_z=False)
            self.progEval = prog
        saved_real = self.d_in[:self.B].clone()
        saved_losses = self.losses.clone()
        self.set_batch(real)
        self._ev_z.copy_(z.to(self.device, torch.float32))
        H.run(self.progEval)
        l = self.losses.tolist()
        self.d_in[:self.B].copy_(saved_real)
        self.losses.copy_(saved_losses)
        return {"d_loss": l[3], "g_loss": l[2]}

    def placement(self) -> List[str]:
        """--log_device_placement lines: every recorded op of the step runs on this rank's HIP
        device; which stream slots / graphs carry it."""
        progs = [("forward+G backward", self.progA), ("D backward", self.progB), ("G weight grads", self.progW),
                 ("optimisers", self.progC)]
        out = ["HIP engine (%s): %d kernels per step, schedule %s, hipGraph %s%s" % (
            self.dtype_name, self.kernel_count(), self._schedule(), "captured" if self.graph_enabled else
            ("requested" if self.graph_requested else "off"),
            ", comm stream for all-reduces" if self.ddp else "")]
        for label, p in progs:
            if p is None:
                continue
            slots = sorted({p.op_info(i)[1] for i in range(p.size())})
            out.append("  %-20s %3d ops on %s, stream slots %s" % (label, p.size(), self.device, slots))
        return out

    def _step_progs(self):
        return [p for p in (self.progA, self.progB, self.progW, self.progC, getattr(self, "progSh", None))
                if p is not None]

    def op_names(self) -> List[str]:
        out = []
        for p in self._step_progs():
            out += [p.name(i) for i in range(p.size())]
        return out

    def kernel_count(self) -> int:
        """Kernel launches per training step (events excluded)."""
        n = 0
        for p in self._step_progs():
            n += sum(1 for i in range(p.size()) if p.op_info(i)[2] == self.ext.OP_LAUNCH)
        return n
