"""Fused HIP training engine: the whole reference DCGAN step on hand-written gfx950 kernels.

The step (``image_train.py:151-158`` semantics) is recorded ONCE into
native ``Program`` objects (``csrc/bindings.cpp``) over statically allocated buffers, then
replayed every step -- optionally captured into hipGraphs so a step is a handful of graph
launches:

  segment A   z ~ U(-1,1) (Philox, device step counter) -> G forward -> D forward on the
              2B batch [real | fake] with per-half BN statistics (= the reference's two
              D calls) -> fused 3-loss BCE -> the g_loss chain back through D(fake)
              (pre-update D weights) into G's backward (G grads final)
  [DDP]       G-gradient all-reduce starts on the comm stream ...
  segment B1  ... while D's backward of d_loss runs (both halves): head + top conv layer
              first, i.e. 76 % of D's gradient bytes (d_h3_conv/w at 64x64) ...
  [DDP]       ... whose all-reduce overlaps ...
  segment B2  ... the rest of D's backward (D grads final); small last all-reduce
  segment C   TF-Adam(G) (its all-reduce is long done), TF-Adam(D), step counter (device
              beta powers, 1/W folded in); each Adam also writes the bf16/fp16 weight mirror
              that the next step's kernels read

G's backward finalises its largest gradient (g_h1/w) LAST and D's backward finalises its
largest FIRST, so running G's backward before D's leaves only a few MB of the 37.8 MB fp32
exchange exposed -- on xGMI rings the bytes, not the number of calls, set the cost.

Layouts: activations NHWC bf16; master weights fp32 in TF layout inside the flat
``ParamSet`` buffers (what the checkpoint writes and DDP reduces); each conv weight also
has bf16 copies packed for the implicit-GEMM kernels ([25][N][Kc]: natural and per-tap
transposed, or an im2col-ordered [N][80] matrix for the 3-channel layers).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import torch

from ..models.config import DCGANConfig, same_pads
from ..models.dcgan import DCGAN
from ..optim.adam import TFAdam
from ..ops import hip as H
from ..parallel import dist as D

RELU, LRELU, TANH, NONE = 1, 2, 3, 0


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())


def _kpad(c: int) -> int:
    return -(-25 * c // 16) * 16


class HipEngine:
    name = "hip"
    dtype_name = "bf16"
    INIT_LOSS_SCALE = 32768.0   # fp16 dynamic loss scaling (TF/Keras LossScaleOptimizer defaults)
    LOSS_SCALE_GROWTH = 2000

    def __init__(self, cfg: DCGANConfig, batch_size: int, device: torch.device, dtype: str = "bf16",
                 seed: int = 0, lr: float = 2e-4, beta1: float = 0.5, zero_debias: bool = False, rank: int = 0,
                 world: int = 1, graph: bool = True, allreduce_dtype: str = "fp32", bucket_mb: float = 32.0,
                 rank_seeded_z: bool = True, **_):
        if dtype not in ("bf16", "fp16"):
            raise ValueError("the HIP engine computes in bf16 or fp16 (fp32 master weights / statistics / "
                             "accumulation); fp32 runs on --engine=reference")
        self.dtype_name = dtype
        self.f16 = dtype == "fp16"
        self.edt = torch.float16 if self.f16 else torch.bfloat16
        if device.type != "cuda":
            raise ValueError("HipEngine needs a GPU")
        self.ext = H.ext()
        self.cfg = cfg
        self.B = int(batch_size)
        self.device = device
        self.rank, self.world = rank, world
        self.seed = int(seed)
        self.rank_seeded_z = bool(rank_seeded_z)  # False only in equivalence tests
        self.lr, self.beta1 = float(lr), float(beta1)
        self.model = DCGAN(cfg, device=device, seed=seed, zero_debias=zero_debias)
        if world > 1:
            D.broadcast_tensors([self.model.g.flat, self.model.d.flat, self.model.g_bn.flat, self.model.d_bn.flat])
        self.opt_d = TFAdam(self.model.d, lr, beta1, power_suffix="")
        self.opt_g = TFAdam(self.model.g, lr, beta1, power_suffix="_1")
        self.opt_d.use_hip = self.opt_g.use_hip = True
        self.grad_d = self.model.d.like()
        self.grad_g = self.model.g.like()
        self._step_host = 0
        self.step_counter = torch.zeros(1, dtype=torch.int64, device=device)  # device global step
        self.graph_requested = bool(graph)
        self.graph_enabled = False
        self._timing = False
        self._graphs: List[Optional[torch.cuda.CUDAGraph]] = []
        self.comm_stream = torch.cuda.Stream(device=device) if world > 1 else None
        self.allreduce_dtype = allreduce_dtype
        self.bucket_mb = bucket_mb
        self._alloc()
        self._build()
        self._repack_weights_now()

    # ------------------------------------------------------------------ buffers
    def _t(self, *shape, dtype=None, zero=False):
        dtype = self.edt if dtype is None else dtype
        f = torch.zeros if zero else torch.empty
        return f(*shape, dtype=dtype, device=self.device)

    def _alloc(self):
        cfg, B = self.cfg, self.B
        B2 = 2 * B
        s = cfg.output_size
        self.gl = cfg.g_layers()
        self.dl = cfg.d_layers()
        t = self._t
        self.z = t(B, cfg.z_dim, dtype=torch.float32)
        self.sample_z = t(B, cfg.z_dim, dtype=torch.float32)
        # ---------------- G
        self.g_h0_pre = t(B, cfg.g_lin_out)
        self.g_h0 = t(B, cfg.g_lin_out)
        self.g_x = {}   # pre-BN deconv outputs
        self.g_a = {}   # activations (post BN+ReLU)
        for L in self.gl[:-1]:
            self.g_x[L.name] = t(B, L.out_hw, L.out_hw, L.cout)
            self.g_a[L.name] = t(B, L.out_hw, L.out_hw, L.cout)
        # ---------------- D input [real | fake]
        self.d_in = t(B2, s, s, cfg.c_dim, zero=True)
        self.real_src = t(B, s, s, cfg.c_dim)
        self.fake = self.d_in[B:]
        self.d_x, self.d_a = {}, {}
        for i, L in enumerate(self.dl):
            if L.bn:
                self.d_x[L.name] = t(B2, L.out_hw, L.out_hw, L.cout)
            self.d_a[L.name] = t(B2, L.out_hw, L.out_hw, L.cout)
        self.kp_d0 = _kpad(cfg.c_dim)
        self.d0_col = t(B2 * self.dl[0].out_hw ** 2, self.kp_d0)
        self.logits = t(B2, dtype=torch.float32)
        self.prob = t(B2, dtype=torch.float32)
        self.losses = t(4, dtype=torch.float32, zero=True)
        self.dl_d = t(B2, dtype=torch.float32)
        self.dl_g = t(B, dtype=torch.float32)
        # ---------------- BN state (fwd): mean/rstd/scale/shift per layer [groups][C]
        self.bn = {}
        for name, C in cfg.g_bn_layers():
            self.bn[name] = {k: t(1, C, dtype=torch.float32) for k in ("mean", "rstd", "scale", "shift")}
        for name, C in cfg.d_bn_layers():
            self.bn[name] = {k: t(2, C, dtype=torch.float32) for k in ("mean", "rstd", "scale", "shift")}
        # ---------------- backward buffers
        self.d_da = {L.name: t(B2, L.out_hw, L.out_hw, L.cout) for L in self.dl}
        self.d_dx = {L.name: t(B2, L.out_hw, L.out_hw, L.cout) for L in self.dl}
        # the g_loss chain back through D(fake) has its own gradient buffers (B rows), so it never
        # shares memory with D's d_loss backward (the two may run concurrently)
        self.gc_da = {L.name: t(B, L.out_hw, L.out_hw, L.cout) for L in self.dl}
        self.gc_dx = {L.name: t(B, L.out_hw, L.out_hw, L.cout) for L in self.dl}
        self.d_head_dx = t(B2, cfg.d_lin_in)
        self.d_head_part = t(16, cfg.d_lin_in, dtype=torch.float32)
        self.img_grad = t(B, s, s, cfg.c_dim)
        self.img_g = t(B, s, s, cfg.c_dim)
        Lg = self.gl[-1]
        self.kp_g = _kpad(cfg.c_dim)
        self.g_last_col = t(B * Lg.in_hw ** 2, self.kp_g)
        self.g_da = {}
        self.g_dx = {}
        for L in self.gl[:-1]:
            self.g_da[L.name] = t(B, L.out_hw, L.out_hw, L.cout)
            self.g_dx[L.name] = t(B, L.out_hw, L.out_hw, L.cout)
        self.g_da0 = t(B, cfg.g_lin_out)
        self.g_dx0 = t(B, cfg.g_lin_out)
        self.coef = {name: t(2, C, 3, dtype=torch.float32) for name, C in cfg.d_bn_layers()}
        self.coef.update({name: t(1, C, 3, dtype=torch.float32) for name, C in cfg.g_bn_layers()})
        self.coef_g = {name: t(1, C, 3, dtype=torch.float32) for name, C in cfg.d_bn_layers()}
        self.small_part = t(64, 16, dtype=torch.float32)
        # ---------------- bf16 weight mirrors: the SAME flat layout as the fp32 masters (TF layouts:
        # HWIO conv, [kh,kw,out,in] deconv), written by the Adam kernel; every conv GEMM reads
        # its weight from here in whichever orientation it needs (igemm3 bkn flag)
        self.wbf_d = self.model.d.like(self.edt)
        self.wbf_g = self.model.g.like(self.edt)
        # fp16: dynamic loss scale state [scale, overflow flag, good steps] (device-resident, so
        # the whole step incl. skip / halve / grow stays inside the captured graphs)
        self.loss_scale = (torch.tensor([self.INIT_LOSS_SCALE, 0.0, 0.0], dtype=torch.float32, device=self.device)
                           if self.f16 else None)

    # ------------------------------------------------------------------ program build
    def _stats_buf(self, key, P, C):
        buf = self._t(P, 2, C, dtype=torch.float32)
        self._keep.append(buf)
        return buf

    def _build(self):
        ext = self.ext
        self._keep: List[torch.Tensor] = []
        self.progA = ext.Program(self.f16)
        self.progB = ext.Program(self.f16)
        self.progC = ext.Program(self.f16)
        self._build_forward(self.progA, update_ema=True, z=self.z, train_z=True, split_d=True)
        self._a_fwd = self.progA.size()  # forward done: D's d_loss backward may start from here
        self._build_gloss_and_g_backward(self.progA)
        self._join(self.progA)
        # opt-in (single process): Adam(G) on the side stream, concurrently with D's backward,
        # joined before Adam(D) / the step counter. Measured on MI355X at 64x64, B=128: 1.634 vs
        # 1.556 ms/step serial -- the memory-bound Adam slows the GEMMs more than it hides.
        self._adam_g_side = (self.world == 1 and not self.f16 and os.environ.get("DCGAN_CONCURRENT_ADAM") == "1")
        if self._adam_g_side:
            ev = self.progA.new_event()
            self.progA.record(ev, 0)
            self.progA.wait(ev, 1)
            self._build_update(self.progA, first=True, stream=1)
        self._build_d_backward_dloss(self.progB)  # sets self._b_split (top layer done)
        self._join(self.progB)
        fused_adam = (not self._adam_g_side and self.world == 1 and not self.f16
                      and os.environ.get("DCGAN_SEPARATE_ADAM") != "1")
        if self._adam_g_side:
            ev = self.progC.new_event()
            self.progC.record(ev, 1)
            self.progC.wait(ev, 0)
            self._c_split = self.progC.size()
            self._build_update(self.progC, first=False)
        elif fused_adam:  # one launch: Adam(G), Adam(D), beta powers, global step
            self._build_update_fused(self.progC)
            self._c_split = self.progC.size()
        else:
            self._build_update(self.progC, first=True)
            self._c_split = self.progC.size()
            self._build_update(self.progC, first=False)
        # opt-in (single process, bf16): Adam(D) on the D chain's stream as soon as D's gradients
        # are final AND the g_loss chain has left D (it reads the pre-update D weights); Adam(G) +
        # the beta-power / step update after the join (see _run_fused). Measured on MI355X at
        # 64x64, B=128: 1.325 vs 1.293 ms/step for the fused two-set Adam after the join -- the
        # memory-bound Adam slows G's backward GEMMs more than it hides
        # (profiles/ab_r1_early_adam_d.txt).
        self._early_adam_d = (self.world == 1 and not self.f16 and not self._adam_g_side
                              and os.environ.get("DCGAN_EARLY_ADAM_D") == "1")
        if self._early_adam_d:
            self.progCd = ext.Program(self.f16)
            self.progCg = ext.Program(self.f16)
            self._build_update_split(self.progCd, self.progCg)
        # D-gradient slice final after segment B1: the top conv layer (+ its BN) and the head,
        # which the ParamSet lays out last
        self._d_top_off = self.model.d.offsets[self.dl[-1].name + "/w"][0]
        self.progCast = ext.Program(self.f16)  # fp32 masters -> bf16/fp16 mirrors (init / checkpoint load)
        for ps, pb in ((self.model.d, self.wbf_d), (self.model.g, self.wbf_g)):
            self.progCast.cast_to_bf16("mirror", _p(ps.flat), 0, _p(pb.flat), ps.flat.numel(), 1.0, 0.0, 0)
        self.progS = None  # sampler program, built lazily
        self.progEval = None

    # ---- helpers
    def _igemm(self, prog, name, mode, A, Bw, C, Bn, Hin, Win, Kc, Hout, Wout, N, pad, out_f32=False, ldc=None,
               cofs=0, bias=None, act=NONE, stats=None, rows_per_group=None, bkn=False, kb_valid=-1, bnb=None,
               stream=0):
        """One conv-shaped GEMM. Bw is a bf16 weight-mirror view; bkn=True reads it as
        [tap][K][N] (D forward, G dgrad, im2col'd layers), else as [tap][N][K]. bnb = (x, y,
        mean, rstd, rows_per_group, act): the epilogue also emits the BN-backward partial sums of
        the layer whose dL/da this GEMM produces (see _dgrad_bnb)."""
        plan = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, rows_per_group, bkn)
        if plan is None:
            raise RuntimeError("no igemm tile for %s (mode %d, N %d, bkn %d)" % (name, mode, N, bkn))
        cfg, splits = plan
        bx = by = bm = br = 0
        brpg = bact = bstore = 0
        if bnb is not None:
            bx, by, bm, br = _p(bnb[0]), _p(bnb[1]), _p(bnb[2]), _p(bnb[3])
            brpg, bact = bnb[4], bnb[5]
            bstore = int(len(bnb) > 6 and bnb[6])
        prog.igemm_ex(name, mode, _p(A), _p(Bw), _p(C), Bn, Hin, Win, Kc, Hout, Wout, N, pad, pad, cfg, int(out_f32),
                      ldc or N, cofs, _p(bias), act, self.cfg.lrelu_leak, _p(stats), stream, int(bkn), kb_valid, splits,
                      bx, by, bm, br, brpg, bact, self.cfg.lrelu_leak, bstore)
        return cfg

    def _dgrad_bnb(self, mode, Bn, Hin, Win, Kc, Hout, Wout, N, bkn, bn_name, x, y, groups, act, group_offset=0):
        """Fused BN-backward statistics for the data-gradient GEMM that writes dL/da of BN layer
        ``bn_name`` (x = its pre-BN input, y = its activation output, same layout as the GEMM
        output). Returns (igemm kwargs, partials, partials per group) or None when no tile keeps
        the real/fake groups apart (odd sizes) -- the BN backward then runs its own stats pass."""
        if os.environ.get("DCGAN_NO_FUSED_BNB") == "1":
            return None
        if mode == 1:
            hq, wq, phases = -(-Hout // 2), -(-Wout // 2), 4
            if Hout % 2 or Wout % 2:
                return None
            M = Bn * hq * wq
        else:
            M, phases = Bn * Hout * Wout, 1
        rpg = M // groups
        plan = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, rpg, bkn)
        if plan is None or N % 8 or not H.bnb_fits(plan[0]):
            return None
        bm, _ = H.tile_of(plan[0])
        P = -(-M // bm) * phases
        part = self._stats_buf(bn_name + ".bwd", P, N)
        st = self.bn[bn_name]
        mean, rstd = st["mean"][group_offset:], st["rstd"][group_offset:]
        kw = dict(stats=part, rows_per_group=rpg, bnb=(x, y, mean, rstd, rpg, act))
        return kw, part, P // groups

    def _dgrad_actb(self, mode, Bn, Hin, Win, Kc, Hout, Wout, N, bkn, name, y, act):
        """Fused activation backward for the data-gradient GEMM that produces dL/da of a layer
        WITHOUT BN: the GEMM stores dx = dL/da * act'(y) directly and emits per-tile partial
        column sums of dx (the bias gradient). Returns (igemm kwargs, partials, #partials) or
        None (no vectorizable tile; the caller runs the separate act backward)."""
        if os.environ.get("DCGAN_NO_FUSED_ACTG") == "1":
            return None
        plan = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, None, bkn)
        if plan is None or N % 8 or not H.bnb_fits(plan[0]):
            return None
        bm, _ = H.tile_of(plan[0])
        if mode == 1:
            M, phases = Bn * (-(-Hout // 2)) * (-(-Wout // 2)), 4
        else:
            M, phases = Bn * Hout * Wout, 1
        P = -(-M // bm) * phases
        part = self._stats_buf(name + ".actb", P, N)
        return dict(stats=part, bnb=(y, y, None, None, 0, act, True)), part, P

    def _deconv_out(self, prog, name, x, w, y, B, L, pad, bias, act):
        """G's output layer: the direct narrow kernel for RGB / gray outputs, else the igemm."""
        if L.cout <= 4 and L.cin % 8 == 0 and L.cin <= 256:
            prog.narrow_deconv(name, _p(x), _p(w), _p(bias), _p(y), B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw,
                               L.cout, pad, act, self.cfg.lrelu_leak, 0)
        else:
            self._igemm(prog, name, 1, x, w, y, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad,
                        bias=bias, act=act)

    def _igemm_stats_tiles(self, mode, Bn, Hin, Win, Kc, Hout, Wout, N, rows_per_group=None, bkn=False):
        if mode == 1:
            M = Bn * (-(-Hout // 2)) * (-(-Wout // 2))
            phases = 4
        else:
            M = Bn * Hout * Wout
            phases = 1
        cfg, _ = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, rows_per_group, bkn)
        bm, _ = H.tile_of(cfg)
        return -(-M // bm) * phases

    def _bn_fwd(self, prog, name, x, y, rows, C, groups, act, part, ppg, update_ema, slot=0, stream=0):
        """BN finalize (+EMA) and apply+act over `groups` row groups whose statistics / EMA
        shadows start at group slot `slot` (D's separate-half passes run groups=1, slot=half)."""
        cfgm = self.cfg
        st = {k: v[slot:] for k, v in self.bn[name].items()}
        bnstate = self.model.d_bn if name.startswith("d_") else self.model.g_bn
        P = self.model.d if name.startswith("d_") else self.model.g
        ema_m = bnstate.mean[name][slot:] if update_ema else None
        ema_v = bnstate.var[name][slot:] if update_ema else None
        tag = name if slot == 0 and groups > 1 or name.startswith("g_") else "%s.%d" % (name, slot)
        prog.bn_finalize(tag + ".fin", _p(part), ppg, groups, C, float(rows // groups), _p(P[name + "/gamma"]),
                         _p(P[name + "/beta"]), cfgm.bn_eps, _p(st["mean"]), _p(st["rstd"]), _p(st["scale"]),
                         _p(st["shift"]), _p(ema_m), _p(ema_v), cfgm.bn_momentum, stream)
        prog.bn_apply_act(tag + ".apply", _p(x), _p(y), _p(st["scale"]), _p(st["shift"]), rows, C,
                          rows // groups, act, cfgm.lrelu_leak, stream)

    @staticmethod
    def _rows_per_block(rows_per_group: int, C: int) -> int:
        """Rows per column-reduction block: a divisor of rows_per_group (blocks never straddle
        a BN group), as large as possible while keeping >= 256 blocks per group (fill the CUs)."""
        for rpb in (256, 128, 64, 32, 16, 8, 4, 2, 1):
            if rows_per_group % rpb == 0 and (rows_per_group // rpb >= 256 or rpb == 1):
                return rpb
        return 1

    # ---- forward
    def _d_forward_half(self, prog, half: int, update_ema: bool, stream: int):
        """D's forward over ONE half of the [real | fake] batch (B rows at row offset half*B):
        the reference's separate D(real) / D(fake) calls (image_train.py:82,85), each with its
        own BN statistics and EMA slot. Used by the split forward, where D(real) runs on the
        side stream concurrently with G's forward."""
        cfg, B = self.cfg, self.B
        Pd, Wd = self.model.d, self.wbf_d
        hs = lambda t: t[half * B:(half + 1) * B]  # noqa: E731  one half of a [2B, ...] buffer
        prev = hs(self.d_in)
        tag = ".r" if half == 0 else ".f"
        for i, L in enumerate(self.dl):
            w = Wd[L.name + "/w"]  # HWIO [5,5,ci,co] = [tap][K][N]
            pad = same_pads(L.in_hw)[0]
            rows = B * L.out_hw ** 2
            if i == 0 and L.cin % 8 != 0:
                col = self.d0_col[half * rows:(half + 1) * rows]
                prog.im2col_s2("d0.im2col" + tag, _p(prev), _p(col), B, L.in_hw, L.in_hw, L.cin, L.out_hw,
                               L.out_hw, pad, pad, self.kp_d0, stream)
                self._igemm(prog, L.name + tag, 2, col, w, hs(self.d_a[L.name]), B, 1, 1, self.kp_d0, L.out_hw,
                            L.out_hw, L.cout, 0, bias=Pd[L.name + "/biases"], act=LRELU, bkn=True,
                            kb_valid=25 * L.cin, stream=stream)
            elif not L.bn:
                self._igemm(prog, L.name + tag, 0, prev, w, hs(self.d_a[L.name]), B, L.in_hw, L.in_hw, L.cin,
                            L.out_hw, L.out_hw, L.cout, pad, bias=Pd[L.name + "/biases"], act=LRELU, bkn=True,
                            stream=stream)
            else:
                P = self._igemm_stats_tiles(0, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, None, True)
                part = self._stats_buf(L.bn + tag, P, L.cout)
                self._igemm(prog, L.name + tag, 0, prev, w, hs(self.d_x[L.name]), B, L.in_hw, L.in_hw, L.cin,
                            L.out_hw, L.out_hw, L.cout, pad, bias=Pd[L.name + "/biases"], stats=part, bkn=True,
                            stream=stream)
                self._bn_fwd(prog, L.bn, hs(self.d_x[L.name]), hs(self.d_a[L.name]), rows, L.cout, 1, LRELU, part,
                             P, update_ema, slot=half, stream=stream)
            prev = hs(self.d_a[L.name])

    def _d0_direct(self) -> bool:
        """D layer 0 forward on the direct conv3 kernel (Cin <= 4, Cout = 64) instead of
        im2col + GEMM; DCGAN_D0_IM2COL=1 keeps the im2col forward."""
        L = self.dl[0]
        return L.cin <= 4 and L.cout == 64 and os.environ.get("DCGAN_D0_IM2COL") != "1"

    def _split_dfwd_ok(self) -> bool:
        """Split forward (opt-in, DCGAN_SPLIT_DFWD=1): D(real) on the side stream beside G's
        forward, D(fake) after G. Measured on MI355X at 64x64, B=128: 1.334 vs 1.321 ms/step
        for the default single D pass over the stacked 2B batch -- G's forward GEMMs already
        fill the CUs, and the half-batch GEMMs run at lower efficiency."""
        if os.environ.get("DCGAN_SPLIT_DFWD") != "1":
            return False
        B = self.B
        for L in self.dl:
            if L.bn and H.igemm_cfg_for(0, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, None,
                                        True) is None:
                return False
        return True

    def _build_forward(self, prog, update_ema: bool, z, train_z: bool, split_d: bool = False):
        cfg, B = self.cfg, self.B
        B2 = 2 * B
        Pg, Pd = self.model.g, self.model.d
        split_d = split_d and self._split_dfwd_ok()
        if prog is self.progA:
            self.split_dfwd = split_d
        if split_d:  # D(real) needs only the real batch and D's weights: start it at once
            ev = prog.new_event()
            prog.record(ev, 0)
            prog.wait(ev, 1)
            self._d_forward_half(prog, 0, update_ema, stream=1)
        zseed = self.seed * 1000003 + 17 + 7919 * self.rank * int(self.rank_seeded_z)
        # train_z: z ~ U(-1,1) generated inside the projection kernel (Philox keyed by the device
        # step counter; DCGAN_SEPARATE_PHILOX=1 keeps the standalone kernel for A/B)
        gen_in_linear = train_z and os.environ.get("DCGAN_SEPARATE_PHILOX") != "1"
        if train_z and not gen_in_linear:
            prog.philox_uniform("z", _p(z), z.numel(), zseed, _p(self.step_counter), 0, -1.0, 1.0, 0)
        # G projection + g_bn0 + relu
        C0 = cfg.g_base_ch
        rows0 = B * cfg.g_base_hw ** 2
        # g_bn0 partial statistics straight from the projection kernel: one partial row per
        # (8-row block of z, spatial position) -- see linear_fwd_kernel
        P0 = -(-B // 8) * (cfg.g_lin_out // C0)
        part0 = self._stats_buf("g_bn0", P0, C0)
        prog.linear_fwd("g_h0_lin", _p(z), _p(Pg["g_h0_lin/Matrix"]), _p(Pg["g_h0_lin/bias"]), _p(self.g_h0_pre),
                        B, cfg.z_dim, cfg.g_lin_out, 0, _p(part0), C0,
                        _p(self.step_counter) if gen_in_linear else 0, zseed if gen_in_linear else 0)
        self._bn_fwd(prog, "g_bn0", self.g_h0_pre, self.g_h0, rows0, C0, 1, RELU, part0, P0, update_ema)
        a_prev = self.g_h0
        Wg, Wd = self.wbf_g, self.wbf_d
        for L in self.gl:
            nat = Wg[L.name + "/w"]  # [5,5,co,ci] = [tap][N][K]
            pad = same_pads(L.out_hw)[0]
            if L.bn:
                P = self._igemm_stats_tiles(1, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout)
                part = self._stats_buf(L.bn, P, L.cout)
                self._igemm(prog, L.name, 1, a_prev, nat, self.g_x[L.name], B, L.in_hw, L.in_hw, L.cin, L.out_hw,
                            L.out_hw, L.cout, pad, bias=Pg[L.name + "/biases"], stats=part)
                rows = B * L.out_hw ** 2
                self._bn_fwd(prog, L.bn, self.g_x[L.name], self.g_a[L.name], rows, L.cout, 1, RELU, part, P,
                             update_ema)
                a_prev = self.g_a[L.name]
            else:  # last: + bias, tanh, written into the fake half of D's input
                self._deconv_out(prog, L.name, a_prev, nat, self.fake, B, L, pad, Pg[L.name + "/biases"], TANH)
        if split_d:  # D(fake) behind G's forward, then join the D(real) branch for the head
            self._d_forward_half(prog, 1, update_ema, stream=0)
            ev = prog.new_event()
            prog.record(ev, 1)
            prog.wait(ev, 0)
            prev = self.d_a[self.dl[-1].name]
        # D forward on [real | fake]
        else:
            prev = self.d_in
        for i, L in enumerate(self.dl if not split_d else ()):
            w = Wd[L.name + "/w"]  # HWIO [5,5,ci,co] = [tap][K][N]
            pad = same_pads(L.in_hw)[0]
            rows = B2 * L.out_hw ** 2
            if i == 0 and self._d0_direct():  # image tile in LDS, no column matrix (conv3.hip)
                prog.conv3_direct("d0.conv3", _p(prev), _p(w), _p(Pd[L.name + "/biases"]), _p(self.d_a[L.name]), B2,
                                  L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad, pad, LRELU,
                                  cfg.lrelu_leak, 0)
            elif i == 0 and L.cin % 8 != 0:
                prog.im2col_s2("d0.im2col", _p(prev), _p(self.d0_col), B2, L.in_hw, L.in_hw, L.cin, L.out_hw,
                               L.out_hw, pad, pad, self.kp_d0, 0)
                self._igemm(prog, L.name, 2, self.d0_col, w, self.d_a[L.name], B2, 1, 1, self.kp_d0, L.out_hw,
                            L.out_hw, L.cout, 0, bias=Pd[L.name + "/biases"], act=LRELU, bkn=True,
                            kb_valid=25 * L.cin)
            elif not L.bn:
                self._igemm(prog, L.name, 0, prev, w, self.d_a[L.name], B2, L.in_hw, L.in_hw, L.cin, L.out_hw,
                            L.out_hw, L.cout, pad, bias=Pd[L.name + "/biases"], act=LRELU, bkn=True)
            else:
                rpg = B * L.out_hw ** 2
                if H.igemm_cfg_for(0, B2, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, rpg, True) is not None:
                    # BN partial statistics straight from the conv epilogue (tiles never straddle
                    # the real/fake boundary)
                    P = self._igemm_stats_tiles(0, B2, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, rpg, True)
                    part = self._stats_buf(L.bn, P, L.cout)
                    self._igemm(prog, L.name, 0, prev, w, self.d_x[L.name], B2, L.in_hw, L.in_hw, L.cin, L.out_hw,
                                L.out_hw, L.cout, pad, bias=Pd[L.name + "/biases"], stats=part, rows_per_group=rpg,
                                bkn=True)
                else:  # odd sizes: no tile divides the group -> separate group-aligned stats pass
                    self._igemm(prog, L.name, 0, prev, w, self.d_x[L.name], B2, L.in_hw, L.in_hw, L.cin, L.out_hw,
                                L.out_hw, L.cout, pad, bias=Pd[L.name + "/biases"], bkn=True)
                    rpb = self._rows_per_block(rpg, L.cout)
                    P = rows // rpb
                    part = self._stats_buf(L.bn, P, L.cout)
                    prog.colstats(L.bn + ".stats", 0, _p(self.d_x[L.name]), 0, 0, 0, 0, 0, 0.0, rows, L.cout, rpb,
                                  rpg, _p(part), 0)
                self._bn_fwd(prog, L.bn, self.d_x[L.name], self.d_a[L.name], rows, L.cout, 2, LRELU, part, P // 2,
                             update_ema)
            prev = self.d_a[L.name]
        lin = cfg.d_lin_name
        if os.environ.get("DCGAN_SEPARATE_LOSS") == "1":
            prog.gemv_head("d_head", _p(prev), _p(Pd[lin + "/Matrix"]), _p(Pd[lin + "/bias"]), _p(self.logits), B2,
                           cfg.d_lin_in, 0)
            prog.gan_loss("loss", _p(self.logits), B, _p(self.losses), _p(self.dl_d), _p(self.dl_g), _p(self.prob), 0,
                          _p(self.loss_scale))
        else:  # head GEMV + the fused 3-loss BCE in its last-arriving block
            prog.gemv_head("d_head+loss", _p(prev), _p(Pd[lin + "/Matrix"]), _p(Pd[lin + "/bias"]), _p(self.logits),
                           B2, cfg.d_lin_in, 0, _p(self.losses), _p(self.dl_d), _p(self.dl_g), _p(self.prob),
                           _p(self.loss_scale))

    # ---- D backward for d_loss (2B rows, both groups) -> all D gradients
    def _build_d_backward_dloss(self, prog):
        cfg, B = self.cfg, self.B
        B2 = 2 * B
        Pd, gD = self.model.d, self.grad_d
        lin = cfg.d_lin_name
        last = self.dl[-1]
        if os.environ.get("DCGAN_NO_HEAD_BWD") == "1":  # A/B: the unfused head backward
            prog.head_wgrad("d_head.wgrad", _p(self.d_a[last.name]), _p(self.dl_d), _p(self.d_head_part), B2,
                            cfg.d_lin_in, 16, _p(gD[lin + "/Matrix"]), _p(gD[lin + "/bias"]), 0)
            prog.head_dgrad("d_head.dgrad", _p(self.dl_d), _p(Pd[lin + "/Matrix"]), _p(self.d_da[last.name]), B2,
                            cfg.d_lin_in, 0)
            fused_next = None
        else:
            fused_next = self._head_bwd(prog, "d_head.bwd", self.d_a[last.name], self.dl_d, self.d_da[last.name],
                                        gD[lin + "/Matrix"], gD[lin + "/bias"], B2, last, 2, 0)
        # fused_next: BN-backward partials emitted by the layer above (head / dgrad GEMM store pass)
        for i in range(len(self.dl) - 1, -1, -1):
            L = self.dl[i]
            rows = B2 * L.out_hw ** 2
            da, a = self.d_da[L.name], self.d_a[L.name]
            dx = self.d_dx[L.name]
            if L.bn:
                self._bn_bwd(prog, L.bn, self.d_x[L.name], da, a, dx, rows, L.cout, 2, LRELU, Pd, gD,
                             self.coef[L.bn], write_param_grads=True, fused=fused_next)
            elif fused_next is not None:  # dx already stored by the upper dgrad GEMM; db from its partials
                part, Pn = fused_next
                prog.sum_partials(L.name + ".dbias", _p(part), Pn, 2 * L.cout, L.cout, _p(gD[L.name + "/biases"]), 0)
            else:  # live bias (no BN after it): db = sum over rows of dx, fused with the act backward
                self._act_bwd_dbias(prog, L.name + ".act_bwd", da, a, dx, rows, L.cout, LRELU, gD[L.name + "/biases"])
            # weight gradient
            src = self.d_in if i == 0 else self.d_a[self.dl[i - 1].name]
            pad = same_pads(L.in_hw)[0]
            if i == 0 and L.cin % 8 != 0:
                if self._d0_direct():  # the forward ran without a column matrix: build it here, off the
                    # critical path (D's chain is the shorter of the two concurrent backward chains)
                    prog.im2col_s2("d0.im2col", _p(self.d_in), _p(self.d0_col), B2, L.in_hw, L.in_hw, L.cin,
                                   L.out_hw, L.out_hw, pad, pad, self.kp_d0, 0)
                self._wgrad(prog, L.name, 2, self.d0_col, 1, 1, self.kp_d0, dx, B2 * L.out_hw ** 2, 1, 1, L.cout, 0,
                            gD[L.name + "/w"])
            else:
                self._wgrad(prog, L.name, 0, src, L.in_hw, L.in_hw, L.cin, dx, B2, L.out_hw, L.out_hw, L.cout, pad,
                            gD[L.name + "/w"])
            if i == len(self.dl) - 1:
                # head + top layer gradients final: DDP splits the segment here so their
                # all-reduce (76 % of D's bytes at 64x64) overlaps the rest of D's backward
                self._join(prog)
                self._b_split = prog.size()
            # data gradient into the previous activation (not needed below layer 0)
            fused_next = None
            if i > 0:
                nat = self.wbf_d[L.name + "/w"]
                P_ = self.dl[i - 1]
                kw = {}
                out = self.d_da[P_.name]
                if P_.bn:
                    r = self._dgrad_bnb(1, B2, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False, P_.bn,
                                        self.d_x[P_.name], self.d_a[P_.name], 2, LRELU)
                    if r is not None:
                        kw, fused_next = r[0], (r[1], r[2])
                else:
                    r = self._dgrad_actb(1, B2, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False, P_.name,
                                         self.d_a[P_.name], LRELU)
                    if r is not None:
                        kw, fused_next, out = r[0], (r[1], r[2]), self.d_dx[P_.name]
                self._igemm(prog, L.name + ".dgrad", 1, dx, nat, out, B2, L.out_hw, L.out_hw, L.cout,
                            L.in_hw, L.in_hw, L.cin, pad, **kw)

    def _act_bwd_dbias(self, prog, name, dy, y, dx, rows, C, act, db):
        """dx = dy * act'(y) and the bias gradient db = column sums of dx: one fused launch
        when the channel count has a kernel variant, else act_bwd + a column-sum pass."""
        leak = self.cfg.lrelu_leak if act == LRELU else 0.0
        fused_ok = os.environ.get("DCGAN_NO_FUSED_ACTB") != "1"
        if fused_ok and (C in (1, 3) or (C % 8 == 0 and C <= 256 and 256 % (C // 8) == 0)):
            prog.act_bwd_dbias(name, _p(dy), _p(y), _p(dx), rows, C, act, leak, _p(db), 0)
        else:
            prog.act_bwd(name, _p(dy), _p(y), _p(dx), dx.numel(), act, leak, 0)
            self._colsum(prog, name + ".dbias", dx, rows, C, db)

    def _head_bwd(self, prog, name, xa, dl, dx, dW, db, R, last, groups, group_offset):
        """D head backward (dx, optional dW / db) with the top BN layer's backward statistics
        fused in: returns (partials, partials per group) for _bn_bwd, or None when the layer
        below the head has no BN / an unsupported channel count (then _bn_bwd runs its own
        statistics pass). group_offset 1 = the fake half only (g_loss chain)."""
        cfg = self.cfg
        Pd = self.model.d
        lin = cfg.d_lin_name
        K = cfg.d_lin_in
        C = last.cout
        ok = bool(last.bn) and C % 64 == 0 and K % C == 0 and os.environ.get("DCGAN_NO_HEAD_STATS") != "1"
        if not ok:
            prog.head_bwd(name, _p(xa), _p(dl), _p(Pd[lin + "/Matrix"]), _p(dx), _p(dW), _p(db), R, K, 0)
            return None
        S = K // C
        part = self._stats_buf(name + ".bnstats", groups * S, C)
        st = self.bn[last.bn]
        r0 = 0 if group_offset == 0 else self.B
        prog.head_bwd(name, _p(xa), _p(dl), _p(Pd[lin + "/Matrix"]), _p(dx), _p(dW), _p(db), R, K, 0,
                      _p(self.d_x[last.name][r0:]), _p(self.d_a[last.name][r0:]), _p(st["mean"][group_offset:]),
                      _p(st["rstd"][group_offset:]), C, R // groups, LRELU, cfg.lrelu_leak, _p(part))
        return part, S

    def _colsum(self, prog, name, x, rows, C, dst):
        if C % 8 == 0:
            rpb = self._rows_per_block(rows, C)
            part = self._stats_buf(name, rows // rpb, C)
            prog.colstats(name, 2, _p(x), 0, 0, 0, 0, 0, 0.0, rows, C, rpb, rows, _p(part), 0)
            prog.sum_partials(name + ".sum", _p(part), rows // rpb, 2 * C, C, _p(dst), 0)
        else:
            blocks = 64
            prog.colsum_small(name, _p(x), rows, C, _p(self.small_part), blocks, 0)
            prog.sum_partials(name + ".sum", _p(self.small_part), blocks, C, C, _p(dst), 0)

    def _wgrad(self, prog, name, mode, G, Hg, Wg, Mc, Dm, Bn, Hd, Wd, Nc, pad, dst):
        K = Bn * Hd * Wd
        taps = 1 if mode == 2 else 25
        # weight gradients may run on a side stream, concurrently with the data-gradient chain
        # on the main stream (both only read dx / the layer input); see _fork
        self._fork(prog)
        if mode == 0:  # 25-tap layers: LDS-DMA pipelined kernel, split-K reduced in-kernel
            plan = H.wgrad3_cfg_for(Mc, Nc, Bn, Hd, Wd, Hg)
            if plan is not None:
                prog.wgrad3(name + ".wgrad", _p(G), Hg, Wg, Mc, _p(Dm), Bn, Hd, Wd, Nc, pad, plan[0], plan[1],
                            _p(dst), 1.0, self.SIDE)
                return
        cfg, splits = H.pick_wgrad(Mc, Nc, K, taps)
        if mode == 0:
            splits = H.wgrad_splits_for(Mc, Nc, Bn, Hd, Wd, Hg) or splits
        slabs = self._t(splits, taps, Mc, Nc, dtype=torch.float32)
        self._keep.append(slabs)
        prog.wgrad(name + ".wgrad", mode, _p(G), Hg, Wg, Mc, _p(Dm), Bn, Hd, Wd, Nc, pad, cfg, splits, _p(slabs),
                   _p(dst), dst.numel(), 1.0, self.SIDE)

    # ---- two-stream structure inside a segment: fork = side waits for main's progress so far,
    # join = main waits for everything queued on side (every segment ends joined, so a segment
    # captures into one hipGraph with parallel branches)
    SIDE = 0

    def _fork(self, prog):
        # Weight gradients stay on the chain's own stream. Running them on a side stream beside
        # the data-gradient chain was measured slower on MI355X (64x64, B=128): 69.4k vs 71.8k
        # img/s with the serial step, and 1.332 vs 1.303 ms/step for G's weight gradients beside
        # the concurrent G chain (profiles/ab_r1_concurrent_wgrad.txt) -- the two backward chains
        # already fill the CUs. The side stream is used by the opt-in split forward only.
        self.SIDE = 0

    def _join(self, prog):
        if getattr(self, "_side_open", False):
            ev = prog.new_event()
            prog.record(ev, 1)
            prog.wait(ev, 0)
            self._side_open = False

    def _bn_bwd(self, prog, name, x, dy, y, dx, rows, C, groups, act, P, grads, coef, write_param_grads,
                stats_key=None, row_offset_groups=None, fused=None):
        """BN + activation backward. fused = (partials, partials per group) when the producing
        data-gradient GEMM already emitted the statistics (else a column-stats pass here)."""
        st = self.bn[name]
        mean, rstd = st["mean"], st["rstd"]
        if row_offset_groups is not None:  # fake-half only (group 1)
            mean = mean[row_offset_groups:row_offset_groups + 1]
            rstd = rstd[row_offset_groups:row_offset_groups + 1]
        rpg = rows // groups
        if fused is not None:
            part, ppg = fused
            Pn = ppg * groups
        else:
            rpb = self._rows_per_block(rpg, C)
            Pn = rows // rpb
            part = self._stats_buf(name + ".bwd", Pn, C)
            prog.colstats(name + ".bwd_stats", 1, _p(x), _p(dy), _p(y), _p(mean), _p(rstd), act,
                          self.cfg.lrelu_leak, rows, C, rpb, rpg, _p(part), 0)
        dg = grads[name + "/gamma"] if write_param_grads else None
        db = grads[name + "/beta"] if write_param_grads else None
        prog.bn_bwd_finalize(name + ".bwd_fin", _p(part), Pn // groups, groups, C, float(rpg), _p(P[name + "/gamma"]),
                             _p(mean), _p(rstd), _p(dg), _p(db), _p(coef), 0)
        prog.bn_bwd_apply(name + ".bwd_apply", _p(dy), _p(y), _p(x), _p(coef), _p(dx), rows, C, rpg, act,
                          self.cfg.lrelu_leak, 0)

    # ---- g_loss back through D(fake) (fake rows only, no D grads) and G backward
    def _build_gloss_and_g_backward(self, prog):
        cfg, B = self.cfg, self.B
        Pd, Pg, gG = self.model.d, self.model.g, self.grad_g
        lin = cfg.d_lin_name
        last = self.dl[-1]
        half = lambda t: t[B:]  # noqa: E731  fake half of a [2B, ...] buffer
        fused_next = self._head_bwd(prog, "g.d_head.dgrad", None, self.dl_g, self.gc_da[last.name], None, None,
                                    B, last, 1, 1)
        for i in range(len(self.dl) - 1, -1, -1):
            L = self.dl[i]
            rows = B * L.out_hw ** 2
            da, a, dx = self.gc_da[L.name], half(self.d_a[L.name]), self.gc_dx[L.name]
            if L.bn:
                self._bn_bwd(prog, L.bn, half(self.d_x[L.name]), da, a, dx, rows, L.cout, 1, LRELU, Pd, None,
                             self.coef_g[L.bn], write_param_grads=False, row_offset_groups=1, fused=fused_next)
            elif fused_next is None:  # (else dx was stored by the upper dgrad GEMM)
                prog.act_bwd("g." + L.name + ".act_bwd", _p(da), _p(a), _p(dx), dx.numel(), LRELU, cfg.lrelu_leak, 0)
            nat = self.wbf_d[L.name + "/w"]
            pad = same_pads(L.in_hw)[0]
            fused_next = None
            if i > 0:
                P_ = self.dl[i - 1]
                kw = {}
                out = self.gc_da[P_.name]
                if P_.bn:
                    r = self._dgrad_bnb(1, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False, P_.bn,
                                        half(self.d_x[P_.name]), half(self.d_a[P_.name]), 1, LRELU, group_offset=1)
                    if r is not None:
                        kw, fused_next = r[0], (r[1], r[2])
                else:
                    r = self._dgrad_actb(1, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False,
                                         "g." + P_.name, half(self.d_a[P_.name]), LRELU)
                    if r is not None:
                        kw, fused_next, out = r[0], (r[1], r[2]), self.gc_dx[P_.name]
                self._igemm(prog, "g." + L.name + ".dgrad", 1, dx, nat, out, B, L.out_hw,
                            L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad, **kw)
            else:
                if L.cin <= 4 and L.cout % 8 == 0 and L.cout <= 256:  # 3-channel image gradient
                    prog.narrow_deconv("g." + L.name + ".dgrad_img", _p(dx), _p(nat), 0, _p(self.img_grad), B,
                                       L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad, NONE, 0.0, 0)
                else:
                    self._igemm(prog, "g." + L.name + ".dgrad_img", 1, dx, nat, self.img_grad, B, L.out_hw,
                                L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad)
        # ---------------- G backward (reads no D state: Adam(D) may run from here on)
        self._a_gd = prog.size()
        n = len(self.gl)
        Lg = self.gl[-1]
        self._act_bwd_dbias(prog, "g_out.tanh_bwd", self.img_grad, self.fake, self.img_g, B * Lg.out_hw ** 2,
                            Lg.cout, TANH, gG[Lg.name + "/biases"])
        a_prev = self.g_a[self.gl[-2].name] if n > 1 else self.g_h0
        da_prev = self.g_da[self.gl[-2].name] if n > 1 else self.g_da0
        x_prev = self.g_x[self.gl[-2].name] if n > 1 else self.g_h0_pre
        bn_prev = self.gl[-2].bn if n > 1 else "g_bn0"
        padL = same_pads(Lg.out_hw)[0]
        wL = self.wbf_g[Lg.name + "/w"]  # [5,5,co,ci] read as [tap][K=co][N=ci]
        if Lg.cout % 8 != 0:
            prog.im2col_s2("g_out.im2col", _p(self.img_g), _p(self.g_last_col), B, Lg.out_hw, Lg.out_hw, Lg.cout,
                           Lg.in_hw, Lg.in_hw, padL, padL, self.kp_g, 0)
            self._wgrad(prog, Lg.name, 2, self.g_last_col, 1, 1, self.kp_g, a_prev, B * Lg.in_hw ** 2, 1, 1, Lg.cin,
                        0, gG[Lg.name + "/w"])
            r = self._dgrad_bnb(2, B, 1, 1, self.kp_g, Lg.in_hw, Lg.in_hw, Lg.cin, True, bn_prev, x_prev, a_prev, 1,
                                RELU)
            fused_next = None
            kw = {}
            if r is not None:
                kw, fused_next = r[0], (r[1], r[2])
            self._igemm(prog, Lg.name + ".dgrad", 2, self.g_last_col, wL, da_prev, B, 1, 1, self.kp_g, Lg.in_hw,
                        Lg.in_hw, Lg.cin, 0, bkn=True, kb_valid=25 * Lg.cout, **kw)
        else:
            self._wgrad(prog, Lg.name, 0, self.img_g, Lg.out_hw, Lg.out_hw, Lg.cout, a_prev, B, Lg.in_hw, Lg.in_hw,
                        Lg.cin, padL, gG[Lg.name + "/w"])
            r = self._dgrad_bnb(0, B, Lg.out_hw, Lg.out_hw, Lg.cout, Lg.in_hw, Lg.in_hw, Lg.cin, True, bn_prev, x_prev,
                                a_prev, 1, RELU)
            fused_next = None
            kw = {}
            if r is not None:
                kw, fused_next = r[0], (r[1], r[2])
            self._igemm(prog, Lg.name + ".dgrad", 0, self.img_g, wL, da_prev, B, Lg.out_hw, Lg.out_hw, Lg.cout,
                        Lg.in_hw, Lg.in_hw, Lg.cin, padL, bkn=True, **kw)
        for j in range(n - 2, -1, -1):
            L = self.gl[j]
            rows = B * L.out_hw ** 2
            x, a, da, dx = self.g_x[L.name], self.g_a[L.name], self.g_da[L.name], self.g_dx[L.name]
            self._bn_bwd(prog, L.bn, x, da, a, dx, rows, L.cout, 1, RELU, Pg, gG, self.coef[L.bn],
                         write_param_grads=True, fused=fused_next)
            src = self.g_a[self.gl[j - 1].name] if j > 0 else self.g_h0
            dsrc = self.g_da[self.gl[j - 1].name] if j > 0 else self.g_da0
            xsrc = self.g_x[self.gl[j - 1].name] if j > 0 else self.g_h0_pre
            bsrc = self.gl[j - 1].bn if j > 0 else "g_bn0"
            pad = same_pads(L.out_hw)[0]
            self._wgrad(prog, L.name, 0, dx, L.out_hw, L.out_hw, L.cout, src, B, L.in_hw, L.in_hw, L.cin, pad,
                        gG[L.name + "/w"])
            r = self._dgrad_bnb(0, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, True, bsrc, xsrc, src, 1,
                                RELU)
            fused_next = None
            kw = {}
            if r is not None:
                kw, fused_next = r[0], (r[1], r[2])
            self._igemm(prog, L.name + ".dgrad", 0, dx, self.wbf_g[L.name + "/w"], dsrc, B, L.out_hw, L.out_hw,
                        L.cout, L.in_hw, L.in_hw, L.cin, pad, bkn=True, **kw)
        # g_bn0 backward + projection gradients
        C0 = cfg.g_base_ch
        rows0 = B * cfg.g_base_hw ** 2
        self._bn_bwd(prog, "g_bn0", self.g_h0_pre, self.g_da0, self.g_h0, self.g_dx0, rows0, C0, 1, RELU, Pg, gG,
                     self.coef["g_bn0"], write_param_grads=True, fused=fused_next)
        prog.linear_wgrad("g_h0_lin.wgrad", _p(self.z), _p(self.g_dx0), _p(gG["g_h0_lin/Matrix"]),
                          _p(gG["g_h0_lin/bias"]), B, cfg.z_dim, cfg.g_lin_out, 0)

    # ---- optimiser (+ bf16 weight mirrors)
    def _build_update(self, prog, first: bool, stream: int = 0):
        """TF-Adam for G (first part) and D + the step counter (last part); each Adam also
        writes the bf16/fp16 mirror the conv GEMMs read. Under DDP the G all-reduce completes
        first (it was issued before D's backward), so Adam(G) runs while D's last bucket is
        still on the wire. fp16: one overflow check over both (all-reduced) gradients gates
        both Adams, so everything runs in the last part."""
        gs = 1.0 / self.world
        od, og = self.opt_d, self.opt_g
        ls = _p(self.loss_scale)
        do_g = (first and not self.f16) or (not first and self.f16)
        do_d = not first
        if self.f16 and do_d:
            prog.nonfinite_check("ls.check_d", _p(self.grad_d.flat), self.grad_d.flat.numel(), ls, 0)
            prog.nonfinite_check("ls.check_g", _p(self.grad_g.flat), self.grad_g.flat.numel(), ls, 0)
        if do_g:
            prog.adam_bf("adam_g", _p(self.model.g.flat), _p(self.wbf_g.flat), _p(self.grad_g.flat), _p(og.m.flat),
                         _p(og.v.flat), _p(og.powers), self.model.g.flat.numel(), og.lr, og.beta1, og.beta2, og.eps,
                         gs, stream, ls)
        if do_d:
            prog.adam_bf("adam_d", _p(self.model.d.flat), _p(self.wbf_d.flat), _p(self.grad_d.flat), _p(od.m.flat),
                         _p(od.v.flat), _p(od.powers), self.model.d.flat.numel(), od.lr, od.beta1, od.beta2, od.eps,
                         gs, 0, ls)
            prog.step_end("step_end", _p(od.powers), _p(og.powers), od.beta1, od.beta2, og.beta1, og.beta2,
                          _p(self.step_counter), 0, ls, self.LOSS_SCALE_GROWTH)

    def _build_update_split(self, prog_d, prog_g):
        """Single-process bf16: TF-Adam(D) alone (prog_d, run beside G's backward), then
        TF-Adam(G) + the beta-power / global-step update (prog_g) -- the same kernels and
        arithmetic as _build_update."""
        od, og = self.opt_d, self.opt_g
        ls = _p(self.loss_scale)
        prog_d.adam_bf("adam_d", _p(self.model.d.flat), _p(self.wbf_d.flat), _p(self.grad_d.flat), _p(od.m.flat),
                       _p(od.v.flat), _p(od.powers), self.model.d.flat.numel(), od.lr, od.beta1, od.beta2, od.eps,
                       1.0, 0, ls)
        prog_g.adam_bf("adam_g", _p(self.model.g.flat), _p(self.wbf_g.flat), _p(self.grad_g.flat), _p(og.m.flat),
                       _p(og.v.flat), _p(og.powers), self.model.g.flat.numel(), og.lr, og.beta1, og.beta2, og.eps,
                       1.0, 0, ls)
        prog_g.step_end("step_end", _p(od.powers), _p(og.powers), od.beta1, od.beta2, og.beta1, og.beta2,
                        _p(self.step_counter), 0, ls, self.LOSS_SCALE_GROWTH)

    def _build_update_fused(self, prog):
        """Single-process bf16: both TF-Adams + the beta-power / global-step update in one launch
        (adam2_kernel), G's buffer first -- the same arithmetic as the separate kernels."""
        od, og = self.opt_d, self.opt_g
        G, Dm = self.model.g, self.model.d
        prog.adam2("adam_gd", _p(G.flat), _p(self.wbf_g.flat), _p(self.grad_g.flat), _p(og.m.flat), _p(og.v.flat),
                   _p(og.powers), G.flat.numel(), og.lr, og.beta1, og.beta2, og.eps, _p(Dm.flat), _p(self.wbf_d.flat),
                   _p(self.grad_d.flat), _p(od.m.flat), _p(od.v.flat), _p(od.powers), Dm.flat.numel(), od.lr,
                   od.beta1, od.beta2, od.eps, 1.0 / self.world, _p(self.step_counter), 0)

    def _repack_weights_now(self):
        H.run(self.progCast)
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ execution
    def _streams(self):
        if not hasattr(self, "_side_stream"):
            self._side_stream = torch.cuda.Stream(device=self.device)
        return [torch.cuda.current_stream(self.device), self._side_stream]

    # Schedules:
    #   "fused"       single process: ONE graph; D's d_loss backward (progB) on its own streams
    #                 concurrently with the g_loss chain + G's backward (progA tail)
    #   "concurrent"  DDP (and the timed single-process step): the same two concurrent chains,
    #                 cut into 6 graphs so the collectives can be issued between them from the
    #                 host: D's top layer + head (76 % of D's bytes) is all-reduced as soon as the
    #                 D chain has produced it, G's gradients as soon as G's backward ends, the
    #                 rest of D's when the D chain ends; Adam(G) / Adam(D) wait for their own
    #                 collectives only
    #   "serial"      DCGAN_SERIAL_DBWD=1: fwd + G backward, then D's backward, as 5 segments
    #                 (G all-reduce overlaps D's backward)
    MAIN, ALT = 0, 1

    def _schedule(self) -> str:
        if self.world == 1 and not self._timing:
            return "fused"
        if os.environ.get("DCGAN_SERIAL_DBWD") == "1" or self._adam_g_side:
            return "serial"
        return "concurrent"

    @property
    def _hybrid(self) -> bool:
        """Concurrent schedule variant (DCGAN_DDP_SCHEDULE=hybrid): only D's top layer + head
        run beside the G chain; the rest of D's backward starts when the G chain ends, so it
        overlaps G's all-reduce (the largest one, 20.5 MB fp32) instead of delaying it."""
        return os.environ.get("DCGAN_DDP_SCHEDULE", "concurrent") == "hybrid"

    def _segments(self):
        """The step as a list of (name, [(program, begin, end)], stream) segments."""
        sch = self._schedule()
        A, B, C = self.progA, self.progB, self.progC
        M = self.MAIN
        if sch == "fused":
            return [("step", [(A, 0, -1), (B, 0, -1), (C, 0, -1)], M)]
        if sch == "serial":
            return [("fwd+G_bwd", [(A, 0, -1)], M), ("D_bwd_top", [(B, 0, self._b_split)], M),
                    ("D_bwd_rest", [(B, self._b_split, -1)], M), ("adam_G", [(C, 0, self._c_split)], M),
                    ("adam_D", [(C, self._c_split, -1)], M)]
        return [("fwd", [(A, 0, self._a_fwd)], M), ("D_bwd_top", [(B, 0, self._b_split)], self.ALT),
                ("G_chain", [(A, self._a_fwd, -1)], M), ("D_bwd_rest", [(B, self._b_split, -1)], self.ALT),
                ("adam_G", [(C, 0, self._c_split)], M), ("adam_D", [(C, self._c_split, -1)], M)]

    def enable_timing(self) -> None:
        """Per-phase GPU timers: the step runs as segments with events between
        them. Call before the first train_step (graphs are captured per segment). Concurrent
        schedule: each phase is reported as ms from the step start to the END of that phase
        (the D and G chains overlap); serial schedule: phase durations."""
        if self._graphs:
            raise RuntimeError("enable_timing() must precede the first train_step")
        self._timing = True
        self._ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(self._segments()) + 1)]

    def phase_times(self) -> Dict[str, float]:
        """Milliseconds of the last step's phases (synchronises on its last event)."""
        if not self._timing:
            return {}
        ev = self._ev
        ev[-1].synchronize()
        segs = self._segments()
        if self._schedule() == "concurrent":
            return {n + "@end": ev[0].elapsed_time(ev[i + 1]) for i, (n, _, _) in enumerate(segs)}
        return {n: ev[i].elapsed_time(ev[i + 1]) for i, (n, _, _) in enumerate(segs)}

    def _concurrent_dbwd(self) -> bool:
        """D's d_loss backward runs on its own streams concurrently with the g_loss chain + G's
        backward (independent buffers; two chains of GEMMs and small latency-bound BN kernels
        fill each other's gaps). Measured on MI355X at 64x64, B=128, single process: 1.32 vs
        1.50 ms/step. DCGAN_SERIAL_DBWD=1 serialises."""
        return self._schedule() != "serial"

    def _alt(self):
        if not hasattr(self, "_alt_streams"):
            self._alt_streams = [torch.cuda.Stream(device=self.device) for _ in range(2)]
        return self._alt_streams

    def _run_fused(self, cs):
        """The "fused" schedule issued onto cs (+ forked alt streams); also what gets captured.
        D's backward starts right after the forward: holding it until the g_loss chain has left
        D (so it overlaps only G's backward) measured 1.314 vs 1.297 ms/step on MI355X."""
        side = self._streams()[1]
        alt = self._alt()
        H.run(self.progA, [cs, side], 0, self._a_fwd)
        fork = torch.cuda.Event()
        fork.record(cs)
        alt[0].wait_event(fork)
        H.run(self.progB, alt)
        if self._early_adam_d:
            H.run(self.progA, [cs, side], self._a_fwd, self._a_gd)   # g_loss chain through D(fake)
            left_d = torch.cuda.Event()
            left_d.record(cs)
            alt[0].wait_event(left_d)
            H.run(self.progCd, alt)                                   # Adam(D) beside G's backward
            H.run(self.progA, [cs, side], self._a_gd, -1)            # G's backward
        else:
            H.run(self.progA, [cs, side], self._a_fwd, -1)
        join = torch.cuda.Event()
        join.record(alt[0])
        cs.wait_event(join)
        H.run(self.progCg if self._early_adam_d else self.progC, [cs, side])

    def _seg(self, i, stream):
        """Run segment i on `stream` (graph replay, or eager replay of its program ranges)."""
        if self.graph_enabled:
            g = self._graphs[i]
            if g is not None:
                with torch.cuda.stream(stream):
                    g.replay()
            return
        _, parts, which = self._segments()[i]
        sec = self._streams()[1] if which == self.MAIN else self._alt()[1]
        for prog, b, e in parts:
            H.run(prog, [stream, sec], b, e)

    def _run_step(self):
        st = self._streams()
        cs = st[0]
        sch = self._schedule()
        if sch == "fused":
            if self.graph_enabled:
                self._seg(0, cs)
            else:
                self._run_fused(cs)
            return
        tick = (lambda i, s: self._ev[i].record(s)) if self._timing else (lambda i, s: None)
        ddp = self.world > 1
        if sch == "concurrent":
            alt = self._alt()[0]
            tick(0, cs)
            self._seg(0, cs)              # z, G fwd, D fwd (real | fake), losses
            tick(1, cs)
            alt.wait_stream(cs)
            self._seg(1, alt)             # D chain: head + top layer gradients
            tick(2, alt)
            if ddp:
                with torch.cuda.stream(alt):
                    self._ar_dtop.launch()
            self._seg(2, cs)              # G chain: g_loss through D(fake), G backward -> grad_g final
            tick(3, cs)
            if ddp:
                with torch.cuda.stream(cs):
                    self._ar_g.launch()
            if self._hybrid:              # the rest of D's backward overlaps G's all-reduce instead
                alt.wait_stream(cs)
            self._seg(3, alt)             # D chain: rest of D's backward -> grad_d final
            tick(4, alt)
            if ddp:
                with torch.cuda.stream(cs):
                    self._ar_g.wait(scale_in_place=False)   # cs waits for dtop + G on the comm stream
            self._seg(4, cs)              # Adam G -> G mirror (overlaps the last D all-reduce)
            tick(5, cs)
            if ddp:
                with torch.cuda.stream(alt):
                    self._ar_drest.launch()
                with torch.cuda.stream(cs):
                    self._ar_drest.wait(scale_in_place=False)
            cs.wait_stream(alt)
            self._seg(5, cs)              # Adam D, step counter, D mirror
            tick(6, cs)
            return
        tick(0, cs)
        self._seg(0, cs)                  # fwd, g_loss chain through D(fake), G backward -> grad_g final
        tick(1, cs)
        if ddp:
            self._ar_g.launch()
        self._seg(1, cs)                  # D backward: head + top layer (overlaps the G all-reduce)
        tick(2, cs)
        if ddp:
            self._ar_dtop.launch()
        self._seg(2, cs)                  # rest of D's backward -> grad_d final
        tick(3, cs)
        if ddp:
            self._ar_drest.launch()
            self._ar_g.wait(scale_in_place=False)
        self._seg(3, cs)                  # Adam G -> G mirror (overlaps the last D all-reduce)
        tick(4, cs)
        if ddp:
            self._ar_dtop.wait(scale_in_place=False)
            self._ar_drest.wait(scale_in_place=False)
        self._seg(4, cs)                  # Adam D, step counter, D mirror
        tick(5, cs)

    def _ensure_comm(self):
        if self.world > 1 and not hasattr(self, "_ar_g"):
            o = self._d_top_off
            cs, mb, wd = self.comm_stream, self.bucket_mb, self.allreduce_dtype
            self._ar_g = D.GradAllReducer(self.grad_g.flat, mb, wd, stream=cs)
            self._ar_dtop = D.GradAllReducer(self.grad_d.flat[o:], mb, wd, stream=cs)
            self._ar_drest = D.GradAllReducer(self.grad_d.flat[:o], mb, wd, stream=cs)

    def _capture(self):
        """Capture each step segment into its own hipGraph (collectives stay outside, issued
        between replays on the comm stream). Capturing does not execute anything; it is
        attempted only after one eager step has loaded every code object, and any failure
        falls back to eager replay of the recorded programs."""
        try:
            torch.cuda.synchronize(self.device)
            graphs = []
            fused = self._schedule() == "fused"
            for name, parts, which in self._segments():
                if all((p.size() if e < 0 else e) <= b for p, b, e in parts):
                    graphs.append(None)  # empty segment (fp16: no separate D update)
                    continue
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    cs = torch.cuda.current_stream(self.device)
                    if fused:
                        self._run_fused(cs)
                    else:
                        sec = self._streams()[1] if which == self.MAIN else self._alt()[1]
                        for prog, b, e in parts:
                            H.run(prog, [cs, sec], b, e)
                graphs.append(g)
            self._graphs = graphs
            return True
        except Exception as e:  # pragma: no cover - depends on runtime
            print("[hip_engine] graph capture failed, running eagerly: %s" % e)
            self._graphs = []
            return False

    def train_step(self) -> None:
        self._ensure_comm()
        if (self.graph_requested and not self.graph_enabled and self._step_host >= 1
                and not getattr(self, "_cap_tried", 0)):
            self._cap_tried = 1
            self.graph_enabled = self._capture()
        self._run_step()
        self._step_host += 1

    @property
    def global_step(self) -> int:
        return int(self.step_counter.item())

    @global_step.setter
    def global_step(self, v: int) -> None:
        self.step_counter.fill_(int(v))

    def set_synthetic_batch(self, real: torch.Tensor) -> None:
        self.set_batch(real)

    def set_batch(self, real: torch.Tensor) -> None:
        """Copy a [B,H,W,C] batch (any float dtype, values already in [-1,1]) into the real half."""
        B = self.B
        if real.shape[0] != B:
            raise ValueError("batch %d != engine batch %d" % (real.shape[0], B))
        self.d_in[:B].copy_(real.to(self.device, non_blocking=True))

    def last_losses(self) -> Dict[str, float]:
        l = self.losses.tolist()
        return {"d_loss_real": l[0], "d_loss_fake": l[1], "g_loss": l[2], "d_loss": l[3]}

    def losses_tensor(self) -> torch.Tensor:
        return self.losses

    def activations(self) -> "Dict[str, torch.Tensor]":
        """Views of the last step's tensors for summaries (no extra compute)."""
        from collections import OrderedDict
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

    # ------------------------------------------------------------------ sampling / eval
    def sampler(self, z: torch.Tensor) -> torch.Tensor:
        """G with inference-mode BN (moving averages) -- distriubted_model.py:131-153."""
        if self.progS is None:
            self._build_sampler()
        self.sample_z.copy_(z.to(self.device, torch.float32))
        H.run(self.progS)
        return self._s_out.float().clone()

    def _build_sampler(self):
        cfg, B = self.cfg, self.B
        prog = self.ext.Program(self.f16)
        Pg = self.model.g
        t = self._t
        self._s_bufs = {}
        h0p, h0 = t(B, cfg.g_lin_out), t(B, cfg.g_lin_out)
        self._s_out = t(B, cfg.output_size, cfg.output_size, cfg.c_dim)
        sc = {name: (t(C, dtype=torch.float32), t(C, dtype=torch.float32)) for name, C in cfg.g_bn_layers()}
        self._s_keep = [h0p, h0, sc]
        bnst = self.model.g_bn
        debias = 1.0
        prog.linear_fwd("s.lin", _p(self.sample_z), _p(Pg["g_h0_lin/Matrix"]), _p(Pg["g_h0_lin/bias"]), _p(h0p), B,
                        cfg.z_dim, cfg.g_lin_out, 0)

        def coef(name, C):
            # zero-debias (if enabled) is applied host-side at build; BN state is read live
            prog.bn_coef_eval("s." + name, C, _p(Pg[name + "/gamma"]), _p(Pg[name + "/beta"]), cfg.bn_eps,
                              _p(bnst.mean[name]), _p(bnst.var[name]), debias, _p(sc[name][0]), _p(sc[name][1]), 0)

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
            prog = self.ext.Program(self.f16)
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

    def sync_state_for_checkpoint(self) -> None:
        torch.cuda.synchronize(self.device)

    def sync_bn_state(self) -> None:
        """Average BN moving averages over ranks (collective; see ReferenceEngine)."""
        D.all_reduce_mean_(self.model.g_bn.flat)
        D.all_reduce_mean_(self.model.d_bn.flat)

    def after_state_load(self) -> None:
        """Call after loading weights/slots from a checkpoint: refresh packed bf16 weights."""
        self._repack_weights_now()

    def op_names(self) -> List[str]:
        out = []
        for p in (self.progA, self.progB, self.progC):
            out += [p.name(i) for i in range(p.size())]
        return out
