"""Fused HIP training engine: the whole reference DCGAN step on hand-written gfx950 kernels.

The step (``image_train.py:151-158`` semantics) is recorded ONCE into
native ``Program`` objects (``csrc/bindings.cpp``) over statically allocated buffers and replayed
every step from C++ (eager, the default) or as hipGraphs:

  progA[:a_fwd]  z ~ U(-1,1) (Philox, device step counter) -> G forward -> D forward on the 2B
                 batch [real | fake] with per-half BN statistics -> fused 3-loss BCE
  progA[a_fwd:]  the g_loss chain back through D(fake) and G's data gradients  -- "G chain"
  progW          G's weight gradients, each tied to the progA position that produces its operand
  progB          D's backward of d_loss, both halves (D grads final)            -- "D chain"
  progC          TF-Adam(G), TF-Adam(D), beta powers, global step (+ 16-bit weight mirrors)

Schedules (``_schedule``), all proven free of cross-stream overlaps by ``schedule_check.py``:
  "fused"       one process: both chains on two streams, G weight gradients on a third, one
                Adam launch after the join
  "concurrent"  DDP default: the chains cut into segments with the gradient collectives issued
                between them on the comm stream (D's top layer first, g_h1's slice as soon as its
                weight gradient exists, the rest as each chain ends; bf16 wire without copies)
  "ddp"         the fused schedule with the collectives inside one hipGraph (native RCCL)
  "serial"      forward + G chain, then the D chain (the G all-reduce under D's backward)

Layouts: activations NHWC in the compute dtype; fp32 master weights in TF layout inside the flat
``ParamSet`` buffers (what checkpoints write and DDP reduces); 16-bit runs keep one mirror of every
weight in the same flat layout, which the GEMMs read in either orientation.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

from ..models.config import DCGANConfig, same_pads
from ..models.dcgan import DCGAN
from ..optim.adam import TFAdam
from ..ops import hip as H
from ..parallel import dist as D
from .hip_aux import HipEngineAux
from .hip_ddp import HipDDPMixin

RELU, LRELU, TANH, NONE = 1, 2, 3, 0
DTYPES = {"bf16": (0, torch.bfloat16), "fp16": (1, torch.float16), "fp32": (2, torch.float32)}
SCHEDULES = ("fused", "ddp", "concurrent", "serial")
DDP_SCHEDULES = ("ddp", "concurrent", "serial")  # schedules that issue the gradient all-reduces


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())


def _kpad(c: int) -> int:
    return -(-25 * c // 16) * 16


_STREAMS: Dict[int, Tuple["torch.cuda.Stream", ...]] = {}


def _engine_streams(dev: torch.device):
    """The side / D-chain streams, created ONCE per device and process: HIP maps each new stream
    onto one of a few hardware queues in turn, so an engine built after many others could get its
    D-chain stream on the main stream's queue -- the two backward chains then serialise (seen as
    28 % slower steps every few engine builds in the in-situ tuner). Shared streams keep the first
    engine's mapping for every later one (engines of a process never run concurrently)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _STREAMS:
        _STREAMS[key] = tuple(torch.cuda.Stream(device=dev) for _ in range(3))
    return _STREAMS[key]


class _TorchExec:
    """Issues a schedule onto real HIP streams (torch.cuda.Stream objects)."""

    def __init__(self, eng: "HipEngine"):
        dev = eng.device
        self.dev = dev
        side, a0, a1 = _engine_streams(dev)
        self.side = side                 # slot 1 of main-stream segments
        self.alt = [a0, a1]              # D chain (+ its slot 1)
        self.comm = eng.comm_stream

    def main(self):
        return torch.cuda.current_stream(self.dev)

    @staticmethod
    def run(prog, streams, begin: int = 0, end: int = -1) -> None:
        H.run(prog, streams, begin, end)

    @staticmethod
    def wait(dst, src) -> None:
        """dst waits for everything queued on src so far."""
        dst.wait_stream(src)

    @staticmethod
    def mark(stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    @staticmethod
    def wait_mark(dst, ev) -> None:
        """dst waits for the work queued on the marked stream up to the mark."""
        dst.wait_event(ev)

    @staticmethod
    def collective(reducer, stream) -> None:
        with torch.cuda.stream(stream):
            reducer.issue()

    @staticmethod
    def replay(graph, stream) -> None:
        with torch.cuda.stream(stream):
            graph.replay()


class HipEngine(HipDDPMixin, HipEngineAux):
    name = "hip"
    dtype_name = "bf16"
    INIT_LOSS_SCALE = 32768.0   # fp16 dynamic loss scaling (TF/Keras LossScaleOptimizer defaults)
    LOSS_SCALE_GROWTH = 2000

    def __init__(self, cfg: DCGANConfig, batch_size: int, device: torch.device, dtype: str = "bf16",
                 seed: int = 0, lr: float = 2e-4, beta1: float = 0.5, zero_debias: bool = False, rank: int = 0,
                 world: int = 1, graph: bool = True, allreduce_dtype: str = "fp32", bucket_mb: float = 32.0,
                 rank_seeded_z: bool = True, schedule: Optional[str] = None, dry_run: bool = False,
                 ddp: Optional[bool] = None, **_):
        if dtype not in DTYPES:
            raise ValueError("HIP engine dtype must be one of %s" % sorted(DTYPES))
        self.dtype_name = dtype
        self.dt, self.edt = DTYPES[dtype]
        self.f16 = dtype == "fp16"
        self.f32 = dtype == "fp32"
        self.dry = bool(dry_run)  # record programs on the CPU for the schedule checker; never runs
        if device.type != "cuda" and not self.dry:
            raise ValueError("HipEngine needs a GPU (dry_run=True only records the step)")
        self.ext = H.ext()
        self.cfg = cfg
        self.B = int(batch_size)
        self.device = device
        self.rank, self.world = rank, world
        # data-parallel path (collectives on the comm stream, segmented step): any W > 1, or a
        # forced one-rank process group (DCGAN_FORCE_DDP=1 / ddp=True: RCCL on a one-GPU box)
        self.ddp = world > 1 or (D.ddp_forced() if ddp is None else bool(ddp))
        self.seed = int(seed)
        self.rank_seeded_z = bool(rank_seeded_z)  # False only in equivalence tests
        self.lr, self.beta1 = float(lr), float(beta1)
        if schedule is None and os.environ.get("DCGAN_SERIAL_DBWD") == "1":
            schedule = "serial"
        if schedule is not None and schedule not in SCHEDULES:
            raise ValueError("schedule must be one of %s" % (SCHEDULES,))
        self._sched_req = schedule
        self.model = DCGAN(cfg, device=device, seed=seed, zero_debias=zero_debias)
        if self.ddp and not self.dry:
            D.broadcast_tensors([self.model.g.flat, self.model.d.flat, self.model.g_bn.flat, self.model.d_bn.flat])
        self.opt_d = TFAdam(self.model.d, lr, beta1, power_suffix="")
        self.opt_g = TFAdam(self.model.g, lr, beta1, power_suffix="_1")
        self.opt_d.use_hip = self.opt_g.use_hip = True
        self.grad_d = self.model.d.like()
        self.grad_g = self.model.g.like()
        self._step_host = 0
        self.step_counter = torch.zeros(1, dtype=torch.int64, device=device)  # device global step
        self.graph_requested = bool(graph) and not self.dry
        self.graph_enabled = False
        self._timing = False
        self._graphs: List[Optional[torch.cuda.CUDAGraph]] = []
        self.comm_stream = torch.cuda.Stream(device=device) if (self.ddp and not self.dry) else None
        self.allreduce_dtype = allreduce_dtype
        # bf16 wire of the segmented DDP step (bf16 engine): flat bf16 gradient images that cast
        # kernels inside the step graphs fill, RCCL reduces in place and Adam reads directly
        self.wire_d = self.wire_g = None
        if self.ddp and allreduce_dtype == "bf16" and self.dt == 0:
            self.wire_d = self.model.d.like(torch.bfloat16)
            self.wire_g = self.model.g.like(torch.bfloat16)
        self.bucket_mb = bucket_mb
        self._exec = None
        self._alloc()
        self._build()
        if not self.dry:
            self._repack_weights_now()

    def _prog(self):
        return self.ext.Program(self.dt, self.dry)

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
        # shares memory with D's d_loss backward (the two run concurrently)
        self.gc_da = {L.name: t(B, L.out_hw, L.out_hw, L.cout) for L in self.dl}
        self.gc_dx = {L.name: t(B, L.out_hw, L.out_hw, L.cout) for L in self.dl}
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
        # one column-sum scratch per chain: the two chains run concurrently
        self.small_part = {"d": t(64, 16, dtype=torch.float32), "g": t(64, 16, dtype=torch.float32)}
        # ---------------- weights the GEMMs read: 16-bit mirrors in the SAME flat layout as the
        # fp32 masters (TF layouts: HWIO conv, [kh,kw,out,in] deconv), written by the Adam kernel;
        # fp32 runs read the masters themselves
        if self.f32:
            self.wbf_d, self.wbf_g = self.model.d, self.model.g
        else:
            self.wbf_d = self.model.d.like(self.edt)
            self.wbf_g = self.model.g.like(self.edt)
        # fp16: dynamic loss scale state [scale, overflow flag, good steps] (device-resident, so
        # the whole step incl. skip / halve / grow stays inside the captured graphs)
        self.loss_scale = (torch.tensor([self.INIT_LOSS_SCALE, 0.0, 0.0], dtype=torch.float32, device=self.device)
                           if self.f16 else None)
        # sampler zero-debias factor 1 / (1 - decay^t) (device scalar, set before each sampler run)
        self._debias = torch.ones(1, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ program build
    def _stats_buf(self, key, P, C):
        buf = self._t(P, 2, C, dtype=torch.float32)
        self._keep.append(buf)
        return buf

    def _build(self):
        self._keep: List[torch.Tensor] = []
        self.progA = self._prog()
        self.progB = self._prog()
        self.progW = self._prog()  # G's weight gradients (see _build_gloss_and_g_backward)
        self._g_w: List[Tuple[int, int]] = []
        self._g_w_layer: List[str] = []
        self._build_forward(self.progA, update_ema=True, z=self.z, train_z=True)
        self._a_fwd = self.progA.size()  # forward done: D's d_loss backward may start from here
        self._build_gloss_and_g_backward(self.progA, self.progW)
        self._build_d_backward_dloss(self.progB)  # sets self._b_split (top layer done)
        # D-gradient slice final after the D chain's first segment: the top conv layer (+ its BN)
        # and the head, which the ParamSet lays out last
        self._d_top_off = self.model.d.offsets[self.dl[-1].name + "/w"][0]
        self._g_cuts = self._g_bucket_cuts()
        self._g_split = self._g_split_plan()
        self._build_shards()
        self._build_updates()  # (after the G split: Adam(G) follows its collectives)
        self.progX, self._wire_ops = self._prog(), {}
        if self.wire_d is not None:  # fp32 gradient slice -> its bf16 wire image, one op per collective
            o = self._d_top_off
            nd, ng = self.grad_d.flat.numel(), self.grad_g.flat.numel()
            lo, hi = self._g_split[3:] if self._g_split is not None else (0, ng)
            for name, src, dst, a, b in (("dtop", self.grad_d, self.wire_d, o, nd), ("drest", self.grad_d, self.wire_d, 0, o),
                                         ("g", self.grad_g, self.wire_g, 0, ng), ("g_a", self.grad_g, self.wire_g, lo, hi),
                                         ("g_b", self.grad_g, self.wire_g, hi, ng), ("g_c", self.grad_g, self.wire_g, 0, lo)):
                if b > a:
                    self._wire_ops[name] = self.progX.size()
                    self.progX.cast_to_bf16("wire." + name, _p(src.flat) + 4 * a, 0, _p(dst.flat) + 2 * a, b - a,
                                            1.0, 0.0, 0)
        self.progCast = self._prog()  # fp32 masters -> 16-bit mirrors (init / checkpoint load)
        if not self.f32:
            for ps, pb in ((self.model.d, self.wbf_d), (self.model.g, self.wbf_g)):
                self.progCast.cast_to_bf16("mirror", _p(ps.flat), 0, _p(pb.flat), ps.flat.numel(), 1.0, 0.0, 0)
        self.progS = None  # sampler program, built lazily
        self.progEval = None
        self.progSum = None

    def _build_updates(self):
        """progC for the current schedule. The one-launch Adam over BOTH models is only used
        where nothing else can be touching D's gradients or weights any more ("fused": after
        the join of the two backward chains). "serial" runs Adam(G) first (progC[:_c_split],
        overlapping D's all-reduces), then Adam(D) + the step counter; "concurrent" -- whose D
        chain ends first -- runs Adam(D) first (overlapping G's all-reduce), then Adam(G) + the
        step counter ("ddp" likewise). fp16: one overflow check gates both, everything in the
        second part."""
        self.progC = self._prog()
        sch = self._schedule()
        if self._sharded():
            self._build_update_sharded(self.progC)
            self._c_split = self._c_split_a = self.progC.size()
        elif sch == "fused" and self.dt == 0:
            self._build_update_fused(self.progC)
            self._c_split = self._c_split_a = self.progC.size()
        elif sch in ("concurrent", "ddp") and not self.f16:
            self._build_update_d_first(self.progC)
        else:
            self._build_update(self.progC, first=True)
            self._c_split = self._c_split_a = self.progC.size()
            self._build_update(self.progC, first=False)


    # ---- helpers
    def _igemm(self, prog, name, mode, A, Bw, C, Bn, Hin, Win, Kc, Hout, Wout, N, pad, out_f32=False, ldc=None,
               cofs=0, bias=None, act=NONE, stats=None, rows_per_group=None, bkn=False, kb_valid=-1, bnb=None,
               stream=0):
        """One conv-shaped GEMM. Bw is a weight view; bkn=True reads it as [tap][K][N] (D
        forward, G dgrad, im2col'd layers), else as [tap][N][K]. bnb = (x, y, mean, rstd,
        rows_per_group, act[, store_g]): the epilogue also emits the BN-backward partial sums of
        the layer whose dL/da this GEMM produces (see _dgrad_bnb)."""
        plan = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, rows_per_group, bkn, dtype=self.dt)
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

    def _stats_tiles(self, mode, Bn, Hin, Win, Kc, Hout, Wout, N, rows_per_group=None, bkn=False):
        """Number of partial-statistics rows a stats-emitting igemm writes (tiles x phases)."""
        if mode == 1:
            M, phases = Bn * (-(-Hout // 2)) * (-(-Wout // 2)), 4
        else:
            M, phases = Bn * Hout * Wout, 1
        plan = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, rows_per_group, bkn, dtype=self.dt)
        if plan is None:
            return None
        bm, _ = H.tile_of(plan[0], self.dt)
        return -(-M // bm) * phases

    def _dgrad_bnb(self, prog, mode, Bn, Hin, Win, Kc, Hout, Wout, N, bkn, bn_name, x, y, groups, act,
                   group_offset=0):
        """Fused BN-backward statistics for the data-gradient GEMM that writes dL/da of BN layer
        ``bn_name`` (x = its pre-BN input, y = its activation output, same layout as the GEMM
        output). Returns (igemm kwargs, partials, partials per group) or None when no tile keeps
        the real/fake groups apart (odd sizes) or in fp32 -- the BN backward then runs its own
        statistics pass. (The BN-backward finalize stays a separate kernel: fusing it into the GEMM
        through a per-workgroup arrival measured slower, profiles/r2/ab_fused_finalize_r2.txt.)"""
        if self.f32:
            return None
        if mode == 1:
            if Hout % 2 or Wout % 2:
                return None
            M, phases = Bn * (Hout // 2) * (Wout // 2), 4
        else:
            M, phases = Bn * Hout * Wout, 1
        rpg = M // groups
        plan = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, rpg, bkn, dtype=self.dt)
        if plan is None or N % 8 or not H.bnb_fits(plan[0]):
            return None
        bm, _ = H.tile_of(plan[0])
        P = -(-M // bm) * phases
        part = self._stats_buf(bn_name + ".bwd", P, N)
        st = self.bn[bn_name]
        mean, rstd = st["mean"][group_offset:], st["rstd"][group_offset:]
        kw = dict(stats=part, rows_per_group=rpg, bnb=(x, y, mean, rstd, rpg, act))
        return kw, part, P // groups

    def _dgrad_actb(self, prog, mode, Bn, Hin, Win, Kc, Hout, Wout, N, bkn, name, y, act):
        """Fused activation backward for the data-gradient GEMM that produces dL/da of a layer
        WITHOUT BN: the GEMM stores dx = dL/da * act'(y) directly and emits per-tile partial
        column sums of dx (the bias gradient). Returns (igemm kwargs, partials, #partials) or
        None (fp32, or no vectorizable tile: the caller runs the separate act backward)."""
        if self.f32:
            return None
        plan = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, None, bkn, dtype=self.dt)
        if plan is None or N % 8 or not H.bnb_fits(plan[0]):
            return None
        bm, _ = H.tile_of(plan[0])
        if mode == 1:
            M, phases = Bn * (-(-Hout // 2)) * (-(-Wout // 2)), 4
        else:
            M, phases = Bn * Hout * Wout, 1
        P = -(-M // bm) * phases
        part = self._stats_buf(name + ".actb", P, N)
        kw = dict(stats=part, bnb=(y, y, None, None, 0, act, True))
        return kw, part, P

    def _deconv_out(self, prog, name, x, w, y, B, L, pad, bias, act):
        """G's output layer: the direct narrow kernel for RGB / gray outputs (16-bit), else the
        implicit GEMM."""
        if not self.f32 and L.cout <= 4 and L.cin % 8 == 0 and L.cin <= 256:
            prog.narrow_deconv(name, _p(x), _p(w), _p(bias), _p(y), B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw,
                               L.cout, pad, act, self.cfg.lrelu_leak, 0)
        else:
            self._igemm(prog, name, 1, x, w, y, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad,
                        bias=bias, act=act)

    def _bn_fwd(self, prog, name, x, y, rows, C, groups, act, part, ppg, update_ema, apply=True):
        """BN finalize (+EMA) and apply+act over `groups` row groups (apply=False: the consumer
        applies it, e.g. the head)."""
        cfgm = self.cfg
        st = self.bn[name]
        bnstate = self.model.d_bn if name.startswith("d_") else self.model.g_bn
        P = self.model.d if name.startswith("d_") else self.model.g
        ema_m = bnstate.mean[name] if update_ema else None
        ema_v = bnstate.var[name] if update_ema else None
        prog.bn_finalize(name + ".fin", _p(part), ppg, groups, C, float(rows // groups), _p(P[name + "/gamma"]),
                         _p(P[name + "/beta"]), cfgm.bn_eps, _p(st["mean"]), _p(st["rstd"]), _p(st["scale"]),
                         _p(st["shift"]), _p(ema_m), _p(ema_v), cfgm.bn_momentum, 0)
        if apply:
            prog.bn_apply_act(name + ".apply", _p(x), _p(y), _p(st["scale"]), _p(st["shift"]), rows, C,
                              rows // groups, act, cfgm.lrelu_leak, 0)

    @staticmethod
    def _rows_per_block(rows_per_group: int, C: int) -> int:
        """Rows per column-reduction block: a divisor of rows_per_group (blocks never straddle
        a BN group), as large as possible while keeping >= 256 blocks per group (fill the CUs)."""
        for rpb in (256, 128, 64, 32, 16, 8, 4, 2, 1):
            if rows_per_group % rpb == 0 and (rows_per_group // rpb >= 256 or rpb == 1):
                return rpb
        return 1

    def _gout_applies_bn(self) -> bool:
        """G's RGB layer (narrow MFMA kernel) applies the BN + ReLU of the layer below itself."""
        L = self.gl[-1]
        return (not self.f32 and len(self.gl) > 1 and bool(self.gl[-2].bn) and L.cout <= 4 and L.cin == 64
                and L.out_hw == 2 * L.in_hw)

    def _head_applies_bn(self) -> bool:
        """The D head GEMV applies the top BN layer's BN + LeakyReLU itself (16-bit builds)."""
        L = self.dl[-1]
        return not self.f32 and bool(L.bn) and L.cout % 8 == 0 and 512 % L.cout == 0 and self.cfg.d_lin_in % 2048 == 0

    def _img_dact(self) -> bool:
        """D layer 0's image gradient (g_loss chain) with G's tanh backward + bias gradient fused
        (narrow.hip DACT): 16-bit, 64-channel D layer 0, <= 4 image channels."""
        L = self.dl[0]
        return not self.f32 and L.cin <= 4 and L.cout == 64 and self.gl[-1].cout == L.cin

    def _g_out_direct(self) -> bool:
        """G's 1..4-channel output layer backward on narrow2.hip (nconv data gradient + nwgrad)."""
        L = self.gl[-1]
        return (not self.f32 and L.cout <= 4 and L.cin == 64
                and self.progA.nwgrad_ok(L.out_hw, L.out_hw, L.in_hw, L.in_hw))

    def _d0_direct(self) -> bool:
        """D layer 0 forward on the direct conv3 kernel (16-bit, Cin <= 4, Cout = 64) instead of
        im2col + GEMM."""
        L = self.dl[0]
        return not self.f32 and L.cin <= 4 and L.cout == 64

    # ---- forward
    def _build_forward(self, prog, update_ema: bool, z, train_z: bool):
        cfg, B = self.cfg, self.B
        B2 = 2 * B
        Pg, Pd = self.model.g, self.model.d
        zseed = self.seed * 1000003 + 17 + 7919 * self.rank * int(self.rank_seeded_z)
        # G projection + g_bn0 + relu; train_z: z ~ U(-1,1) generated inside the projection kernel
        # (Philox keyed by the device step counter); g_bn0 partial statistics straight from it:
        # one partial row per (8-row block of z, spatial position) -- see linear_fwd_kernel
        C0 = cfg.g_base_ch
        rows0 = B * cfg.g_base_hw ** 2
        P0 = -(-B // 8) * (cfg.g_lin_out // C0)
        part0 = self._stats_buf("g_bn0", P0, C0)
        prog.linear_fwd("g_h0_lin", _p(z), _p(Pg["g_h0_lin/Matrix"]), _p(Pg["g_h0_lin/bias"]), _p(self.g_h0_pre),
                        B, cfg.z_dim, cfg.g_lin_out, 0, _p(part0), C0,
                        _p(self.step_counter) if train_z else 0, zseed if train_z else 0)
        self._bn_fwd(prog, "g_bn0", self.g_h0_pre, self.g_h0, rows0, C0, 1, RELU, part0, P0, update_ema)
        a_prev = self.g_h0
        Wg, Wd = self.wbf_g, self.wbf_d
        for L in self.gl:
            nat = Wg[L.name + "/w"]  # [5,5,co,ci] = [tap][N][K]
            pad = same_pads(L.out_hw)[0]
            if L.bn:
                P = self._stats_tiles(1, B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout)
                part = self._stats_buf(L.bn, P, L.cout)
                rows = B * L.out_hw ** 2
                self._igemm(prog, L.name, 1, a_prev, nat, self.g_x[L.name], B, L.in_hw, L.in_hw, L.cin, L.out_hw,
                            L.out_hw, L.cout, pad, bias=Pg[L.name + "/biases"], stats=part)
                out_applies = L is self.gl[-2] and self._gout_applies_bn()
                self._bn_fwd(prog, L.bn, self.g_x[L.name], self.g_a[L.name], rows, L.cout, 1, RELU, part, P,
                             update_ema, apply=not out_applies)
                a_prev = self.g_a[L.name]
            elif self._gout_applies_bn():
                # RGB layer: the lower layer's BN apply + ReLU in its halo staging (writes that
                # activation), + bias, tanh into the fake half of D's input
                Lp = self.gl[-2]
                st = self.bn[Lp.bn]
                prog.narrow_deconv_bnin(L.name + "+bn_apply", _p(self.g_x[Lp.name]), _p(nat), _p(Pg[L.name + "/biases"]),
                                        _p(self.fake), B, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, pad,
                                        TANH, cfg.lrelu_leak, _p(st["scale"]), _p(st["shift"]), RELU, cfg.lrelu_leak,
                                        _p(self.g_a[Lp.name]), 0)
            else:  # last: + bias, tanh, written into the fake half of D's input
                self._deconv_out(prog, L.name, a_prev, nat, self.fake, B, L, pad, Pg[L.name + "/biases"], TANH)
        # D forward on [real | fake]
        prev = self.d_in
        for i, L in enumerate(self.dl):
            w = Wd[L.name + "/w"]  # HWIO [5,5,ci,co] = [tap][K][N]
            pad = same_pads(L.in_hw)[0]
            rows = B2 * L.out_hw ** 2
            if i == 0 and self._d0_direct():  # persistent direct MFMA conv, no column matrix (narrow2.hip)
                prog.nconv("d0.nconv", _p(prev), _p(w), _p(Pd[L.name + "/biases"]), _p(self.d_a[L.name]), B2,
                           L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, pad, pad, LRELU, cfg.lrelu_leak,
                           H.nconv_grid(prog, B2, L.out_hw, L.out_hw), 0, 0, 0, 0, 0, 0.0, 0, 0)
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
                P = self._stats_tiles(0, B2, L.in_hw, L.in_hw, L.cin, L.out_hw, L.out_hw, L.cout, rpg, True)
                if P is not None:
                    # BN partial statistics straight from the conv epilogue (tiles never straddle
                    # the real/fake boundary)
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
                head_bn = i == len(self.dl) - 1 and self._head_applies_bn()
                self._bn_fwd(prog, L.bn, self.d_x[L.name], self.d_a[L.name], rows, L.cout, 2, LRELU, part, P // 2,
                             update_ema, apply=not head_bn)
            prev = self.d_a[L.name]
        lin = cfg.d_lin_name
        last = self.dl[-1]
        if last.bn and self._head_applies_bn():
            # head GEMV with the top BN layer's apply + LeakyReLU fused (writes its activation) + the
            # fused 3-loss BCE in its last-arriving block
            st = self.bn[last.bn]
            prog.gemv_head_bn("d_head+bn_apply+loss", _p(self.d_x[last.name]), _p(Pd[lin + "/Matrix"]),
                              _p(Pd[lin + "/bias"]), _p(self.logits), B2, cfg.d_lin_in, 0, _p(self.losses),
                              _p(self.dl_d), _p(self.dl_g), _p(self.prob), _p(self.loss_scale), _p(st["scale"]),
                              _p(st["shift"]), last.cout, B, LRELU, cfg.lrelu_leak, _p(self.d_a[last.name]))
        else:
            # head GEMV + the fused 3-loss BCE in its last-arriving block
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
                part, Pn = fused_next[0], fused_next[1]
                prog.sum_partials(L.name + ".dbias", _p(part), Pn, 2 * L.cout, L.cout, _p(gD[L.name + "/biases"]), 0)
            else:  # live bias (no BN after it): db = sum over rows of dx, fused with the act backward
                self._act_bwd_dbias(prog, L.name + ".act_bwd", da, a, dx, rows, L.cout, LRELU, gD[L.name + "/biases"],
                                    "d")

            def emit_wgrad(i=i, L=L, dx=dx):
                src = self.d_in if i == 0 else self.d_a[self.dl[i - 1].name]
                pad = same_pads(L.in_hw)[0]
                ws = 0
                if i == 0 and self._d0_direct() and prog.nwgrad_ok(L.in_hw, L.in_hw, L.out_hw, L.out_hw):
                    # image window staged per workgroup, no column matrix (narrow2.hip nwgrad)
                    prog.nwgrad(L.name + ".nwgrad", _p(self.d_in), B2, L.in_hw, L.in_hw, L.cin, _p(dx), L.out_hw,
                                L.out_hw, pad, _p(gD[L.name + "/w"]), ws)
                elif i == 0 and L.cin % 8 != 0:
                    if self._d0_direct():  # the forward ran without a column matrix: build it here
                        prog.im2col_s2("d0.im2col", _p(self.d_in), _p(self.d0_col), B2, L.in_hw, L.in_hw, L.cin,
                                       L.out_hw, L.out_hw, pad, pad, self.kp_d0, ws)
                    self._wgrad(prog, L.name, 2, self.d0_col, 1, 1, self.kp_d0, dx, B2 * L.out_hw ** 2, 1, 1, L.cout, 0,
                                gD[L.name + "/w"], stream=ws)
                else:
                    self._wgrad(prog, L.name, 0, src, L.in_hw, L.in_hw, L.cin, dx, B2, L.out_hw, L.out_hw, L.cout, pad,
                                gD[L.name + "/w"], stream=ws)
                if i == len(self.dl) - 1:
                    # head + top layer gradients final: DDP splits the segment here so their
                    # all-reduce (76 % of D's bytes at 64x64) overlaps the rest of D's backward
                    self._b_split = prog.size()

            def emit_dgrad(i=i, L=L, dx=dx):
                fused = None
                pad = same_pads(L.in_hw)[0]
                if i > 0:
                    nat = self.wbf_d[L.name + "/w"]
                    P_ = self.dl[i - 1]
                    kw = {}
                    out = self.d_da[P_.name]
                    if P_.bn:
                        r = self._dgrad_bnb(prog, 1, B2, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False,
                                            P_.bn, self.d_x[P_.name], self.d_a[P_.name], 2, LRELU)
                        if r is not None:
                            kw, fused = r[0], (r[1], r[2])
                    else:
                        r = self._dgrad_actb(prog, 1, B2, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False,
                                             P_.name, self.d_a[P_.name], LRELU)
                        if r is not None:
                            kw, fused, out = r[0], (r[1], r[2]), self.d_dx[P_.name]
                    self._igemm(prog, L.name + ".dgrad", 1, dx, nat, out, B2, L.out_hw, L.out_hw, L.cout,
                                L.in_hw, L.in_hw, L.cin, pad, **kw)
                return fused

            # weight gradient, then data gradient (dgrad-first measured neutral:
            # profiles/r2/ab_d_dgrad_first_r2.txt)
            emit_wgrad()
            fused_next = emit_dgrad()
            if i == len(self.dl) - 1:
                self._b_top_dgrad = prog.size()  # the D chain's last read of the top layer's kernel

    def _w_mark(self, prog, progw, begin: int, layer: str) -> None:
        """progW[begin:] (`layer`'s weight gradient) needs progA up to its current end."""
        if progw.size() > begin:
            self._g_w.append((prog.size(), progw.size()))
            self._g_w_layer.append(layer)

    def _act_bwd_dbias(self, prog, name, dy, y, dx, rows, C, act, db, chain):
        """dx = dy * act'(y) and the bias gradient db = column sums of dx: one fused launch
        when the channel count has a kernel variant, else act_bwd + a column-sum pass."""
        leak = self.cfg.lrelu_leak if act == LRELU else 0.0
        if C in (1, 3) or (C % 8 == 0 and C <= 256 and 256 % (C // 8) == 0):
            prog.act_bwd_dbias(name, _p(dy), _p(y), _p(dx), rows, C, act, leak, _p(db), 0)
        else:
            prog.act_bwd(name, _p(dy), _p(y), _p(dx), dx.numel(), act, leak, 0)
            self._colsum(prog, name + ".dbias", dx, rows, C, db, chain)

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
        if not (bool(last.bn) and C % 64 == 0 and K % C == 0):
            prog.head_bwd(name, _p(xa), _p(dl), _p(Pd[lin + "/Matrix"]), _p(dx), _p(dW), _p(db), R, K, 0)
            return None
        S = K // C
        # row splits: RS x the workgroups of one-per-64-columns (the head's R rows are few)
        RS = 2  # (A/B 1 / 2 / 4 splits: 2 best, profiles/r2/ab_head_nconv_nwgrad_r2.txt)
        while RS > 1 and (R % RS or (R // groups) % (R // RS)):
            RS //= 2
        part = self._stats_buf(name + ".bnstats", groups * RS * S, C)
        st = self.bn[last.bn]
        r0 = 0 if group_offset == 0 else self.B
        prog.head_bwd_rs(name, _p(xa), _p(dl), _p(Pd[lin + "/Matrix"]), _p(dx), _p(dW), _p(db), R, K, 0,
                         _p(self.d_x[last.name][r0:]), _p(self.d_a[last.name][r0:]), _p(st["mean"][group_offset:]),
                         _p(st["rstd"][group_offset:]), C, R // groups, LRELU, cfg.lrelu_leak, _p(part), RS)
        return part, RS * S

    def _colsum(self, prog, name, x, rows, C, dst, chain):
        if C % 8 == 0:
            rpb = self._rows_per_block(rows, C)
            part = self._stats_buf(name, rows // rpb, C)
            prog.colstats(name, 2, _p(x), 0, 0, 0, 0, 0, 0.0, rows, C, rpb, rows, _p(part), 0)
            prog.sum_partials(name + ".sum", _p(part), rows // rpb, 2 * C, C, _p(dst), 0)
        else:
            blocks = 64
            sp = self.small_part[chain]
            prog.colsum_small(name, _p(x), rows, C, _p(sp), blocks, 0)
            prog.sum_partials(name + ".sum", _p(sp), blocks, C, C, _p(dst), 0)

    def _wgrad(self, prog, name, mode, G, Hg, Wg, Mc, Dm, Bn, Hd, Wd, Nc, pad, dst, stream=0):
        """Weight gradient dst [25][Mc][Nc] (fp32): wgrad3 / wgrad5 (16-bit, 25-tap layers, split-K
        reduced on the device, deterministic), else the first-generation slab kernel + reduce."""
        K = Bn * Hd * Wd
        taps = 1 if mode == 2 else 25
        if mode == 0 and not self.f32:  # 25-tap layers: LDS-DMA pipelined kernel, split-K reduced in-kernel
            plan = H.wgrad3_cfg_for(Mc, Nc, Bn, Hd, Wd, Hg)
            if plan is not None:
                prog.wgrad3(name + ".wgrad", _p(G), Hg, Wg, Mc, _p(Dm), Bn, Hd, Wd, Nc, pad, plan[0], plan[1],
                            _p(dst), 1.0, stream)
                return
        cfg, splits = H.pick_wgrad(Mc, Nc, K, taps, dtype=self.dt)
        if mode == 0 and not self.f32:
            splits = H.wgrad_splits_for(Mc, Nc, Bn, Hd, Wd, Hg) or splits
        slabs = self._t(splits, taps, Mc, Nc, dtype=torch.float32)
        self._keep.append(slabs)
        prog.wgrad(name + ".wgrad", mode, _p(G), Hg, Wg, Mc, _p(Dm), Bn, Hd, Wd, Nc, pad, cfg, splits, _p(slabs),
                   _p(dst), dst.numel(), 1.0, stream)

    def _bn_bwd(self, prog, name, x, dy, y, dx, rows, C, groups, act, P, grads, coef, write_param_grads,
                row_offset_groups=None, fused=None):
        """BN + activation backward. fused = (partials, partials per group) when the producing
        data-gradient GEMM already emitted the statistics (else a column-stats pass here)."""
        st = self.bn[name]
        mean, rstd = st["mean"], st["rstd"]
        if row_offset_groups is not None:  # fake-half only (group 1)
            mean = mean[row_offset_groups:row_offset_groups + 1]
            rstd = rstd[row_offset_groups:row_offset_groups + 1]
        rpg = rows // groups
        if fused is not None:
            part, ppg = fused[0], fused[1]
            Pn = ppg * groups
        else:
            rpb = self._rows_per_block(rpg, C)
            Pn = rows // rpb
            part = self._stats_buf(name + ".bwd", Pn, C)
            prog.colstats(name + ".bwd_stats", 1, _p(x), _p(dy), _p(y), _p(mean), _p(rstd), act,
                          self.cfg.lrelu_leak, rows, C, rpb, rpg, _p(part), 0)
        dg = grads[name + "/gamma"] if write_param_grads else None
        db = grads[name + "/beta"] if write_param_grads else None
        prog.bn_bwd_finalize(name + ".bwd_fin", _p(part), Pn // groups, groups, C, float(rpg),
                             _p(P[name + "/gamma"]), _p(mean), _p(rstd), _p(dg), _p(db), _p(coef), 0)
        prog.bn_bwd_apply(name + ".bwd_apply", _p(dy), _p(y), _p(x), _p(coef), _p(dx), rows, C, rpg, act,
                          self.cfg.lrelu_leak, 0)

    # ---- g_loss back through D(fake) (fake rows only, no D grads) and G backward
    def _build_gloss_and_g_backward(self, prog, progw):
        """progA: g_loss back through D(fake), then G's data-gradient chain; progw: G's weight
        gradients, each recorded with the progA position it needs (self._g_w). Under the fused
        schedule they run on the D chain's stream once that chain is done, beside the G
        data-gradient chain (which then has nothing else on its critical path)."""
        cfg, B = self.cfg, self.B
        Pd, Pg, gG = self.model.d, self.model.g, self.grad_g
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
                    r = self._dgrad_bnb(prog, 1, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False,
                                        P_.bn, half(self.d_x[P_.name]), half(self.d_a[P_.name]), 1, LRELU,
                                        group_offset=1)
                    if r is not None:
                        kw, fused_next = r[0], (r[1], r[2])
                else:
                    r = self._dgrad_actb(prog, 1, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, False,
                                         "g." + P_.name, half(self.d_a[P_.name]), LRELU)
                    if r is not None:
                        kw, fused_next, out = r[0], (r[1], r[2]), self.gc_dx[P_.name]
                self._igemm(prog, "g." + L.name + ".dgrad", 1, dx, nat, out, B, L.out_hw,
                            L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad, **kw)
            else:
                if self._img_dact():
                    # image gradient with G's tanh backward fused (dL/d(G pre-activation) straight out)
                    # + the G output bias gradient from its per-workgroup column sums
                    Lg = self.gl[-1]
                    prog.narrow_deconv_dact("g." + L.name + ".dgrad_img+tanh_bwd", _p(dx), _p(nat), _p(self.img_g),
                                            _p(self.fake), B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin,
                                            pad, TANH, 0.0, _p(self.grad_g[Lg.name + "/biases"]), 0)
                elif not self.f32 and L.cin <= 4 and L.cout % 8 == 0 and L.cout <= 256:  # 3-channel image gradient
                    prog.narrow_deconv("g." + L.name + ".dgrad_img", _p(dx), _p(nat), 0, _p(self.img_grad), B,
                                       L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad, NONE, 0.0, 0)
                else:
                    self._igemm(prog, "g." + L.name + ".dgrad_img", 1, dx, nat, self.img_grad, B, L.out_hw,
                                L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, pad)
        self._build_g_backward(prog, progw)

    def _build_g_backward(self, prog, progw):
        """G's backward from the image gradient img_g (G's tanh backward already applied when the
        image-gradient kernel fused it): data gradients into prog, weight gradients into progw."""
        cfg, B = self.cfg, self.B
        Pg, gG = self.model.g, self.grad_g
        self._a_gd_end = prog.size()  # the g_loss chain is done with D's weights / BN parameters
        n = len(self.gl)
        Lg = self.gl[-1]
        if not self._img_dact():  # (else fused into the image-gradient kernel above)
            self._act_bwd_dbias(prog, "g_out.tanh_bwd", self.img_grad, self.fake, self.img_g, B * Lg.out_hw ** 2,
                                Lg.cout, TANH, gG[Lg.name + "/biases"], "g")
        a_prev = self.g_a[self.gl[-2].name] if n > 1 else self.g_h0
        da_prev = self.g_da[self.gl[-2].name] if n > 1 else self.g_da0
        x_prev = self.g_x[self.gl[-2].name] if n > 1 else self.g_h0_pre
        bn_prev = self.gl[-2].bn if n > 1 else "g_bn0"
        padL = same_pads(Lg.out_hw)[0]
        wL = self.wbf_g[Lg.name + "/w"]  # [5,5,co,ci] read as [tap][K=co][N=ci]
        if self._g_out_direct():
            # narrow2.hip: the data gradient is the stride-2 conv of the image gradient with the
            # [5,5,co,ci] = HWIO[5,5,3,64] weight (nconv, BN-backward statistics of the layer below
            # fused), the weight gradient reads the image gradient's window directly (nwgrad)
            # persistent grid (one workgroup per tile measured the same beside the D chain)
            grid = H.nconv_grid(prog, B, Lg.in_hw, Lg.in_hw)
            part = self._stats_buf(bn_prev + ".bwd", grid, Lg.cin)
            st = self.bn[bn_prev]
            w0 = progw.size()
            progw.nwgrad(Lg.name + ".nwgrad", _p(self.img_g), B, Lg.out_hw, Lg.out_hw, Lg.cout, _p(a_prev), Lg.in_hw,
                         Lg.in_hw, padL, _p(gG[Lg.name + "/w"]), 0)
            self._w_mark(prog, progw, w0, Lg.name)
            prog.nconv(Lg.name + ".dgrad", _p(self.img_g), _p(wL), 0, _p(da_prev), B, Lg.out_hw, Lg.out_hw, Lg.cout,
                       Lg.in_hw, Lg.in_hw, padL, padL, NONE, 0.0, grid, _p(x_prev), _p(a_prev), _p(st["mean"]),
                       _p(st["rstd"]), RELU, cfg.lrelu_leak, _p(part), 0)
            fused_next = (part, grid, {})
        elif Lg.cout % 8 != 0:
            prog.im2col_s2("g_out.im2col", _p(self.img_g), _p(self.g_last_col), B, Lg.out_hw, Lg.out_hw, Lg.cout,
                           Lg.in_hw, Lg.in_hw, padL, padL, self.kp_g, 0)
            w0 = progw.size()
            self._wgrad(progw, Lg.name, 2, self.g_last_col, 1, 1, self.kp_g, a_prev, B * Lg.in_hw ** 2, 1, 1, Lg.cin,
                        0, gG[Lg.name + "/w"])
            self._w_mark(prog, progw, w0, Lg.name)
            r = self._dgrad_bnb(prog, 2, B, 1, 1, self.kp_g, Lg.in_hw, Lg.in_hw, Lg.cin, True, bn_prev, x_prev,
                                a_prev, 1, RELU)
            fused_next = None
            kw = {}
            if r is not None:
                kw, fused_next = r[0], (r[1], r[2])
            self._igemm(prog, Lg.name + ".dgrad", 2, self.g_last_col, wL, da_prev, B, 1, 1, self.kp_g, Lg.in_hw,
                        Lg.in_hw, Lg.cin, 0, bkn=True, kb_valid=25 * Lg.cout, **kw)
        else:
            w0 = progw.size()
            self._wgrad(progw, Lg.name, 0, self.img_g, Lg.out_hw, Lg.out_hw, Lg.cout, a_prev, B, Lg.in_hw, Lg.in_hw,
                        Lg.cin, padL, gG[Lg.name + "/w"])
            self._w_mark(prog, progw, w0, Lg.name)
            r = self._dgrad_bnb(prog, 0, B, Lg.out_hw, Lg.out_hw, Lg.cout, Lg.in_hw, Lg.in_hw, Lg.cin, True, bn_prev,
                                x_prev, a_prev, 1, RELU)
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
            w0 = progw.size()
            self._wgrad(progw, L.name, 0, dx, L.out_hw, L.out_hw, L.cout, src, B, L.in_hw, L.in_hw, L.cin, pad,
                        gG[L.name + "/w"])
            self._w_mark(prog, progw, w0, L.name)
            r = self._dgrad_bnb(prog, 0, B, L.out_hw, L.out_hw, L.cout, L.in_hw, L.in_hw, L.cin, True, bsrc, xsrc,
                                src, 1, RELU)
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


    # ---- optimiser (+ 16-bit weight mirrors)
    def _build_update(self, prog, first: bool):
        """TF-Adam for G (first part) and D + the step counter (last part); each Adam also
        writes the 16-bit mirror the conv GEMMs read (fp32: none, the GEMMs read the masters).
        Under DDP the G all-reduce completes first (it was issued before D's backward ends), so
        Adam(G) runs while D's last bucket is still on the wire. fp16: one overflow check over
        both (all-reduced) gradients gates both Adams, so everything runs in the last part."""
        gs = 1.0 / self.world
        od, og = self.opt_d, self.opt_g
        ls = _p(self.loss_scale)
        do_g = (first and not self.f16) or (not first and self.f16)
        do_d = not first
        mg = 0 if self.f32 else _p(self.wbf_g.flat)
        md = 0 if self.f32 else _p(self.wbf_d.flat)
        if self.f16 and do_d:
            prog.nonfinite_check("ls.check_d", _p(self.grad_d.flat), self.grad_d.flat.numel(), ls, 0)
            prog.nonfinite_check("ls.check_g", _p(self.grad_g.flat), self.grad_g.flat.numel(), ls, 0)
        if do_g:
            prog.adam_bf("adam_g", _p(self.model.g.flat), mg, _p(self.grad_g.flat), _p(og.m.flat),
                         _p(og.v.flat), _p(og.powers), self.model.g.flat.numel(), og.lr, og.beta1, og.beta2, og.eps,
                         gs, 0, ls)
        if do_d:
            prog.adam_bf("adam_d", _p(self.model.d.flat), md, _p(self.grad_d.flat), _p(od.m.flat),
                         _p(od.v.flat), _p(od.powers), self.model.d.flat.numel(), od.lr, od.beta1, od.beta2, od.eps,
                         gs, 0, ls)
            prog.step_end("step_end", _p(od.powers), _p(og.powers), od.beta1, od.beta2, og.beta1, og.beta2,
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
        if self.progCast.size():
            H.run(self.progCast)
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ execution
    MAIN, ALT = 0, 1
    # G's weight gradients off the G chain's stream (fused schedule; where: _gw_place): None = by
    # image size. Round 2, behind the D chain (profiles/r2/ab_g_wgrad_after_d_chain_r2.txt): 64x64
    # 1.105 vs 1.13 ms, 28x28 even, 128x128 5.84 vs 5.70 ms, 256x256 106.2 vs 104.6 ms -- at the
    # larger sizes the D chain (2B rows of the bigger images) is the longer one already
    G_WGRAD_ON_D_STREAM: Optional[bool] = None

    def _g_wgrad_on_d_stream(self) -> bool:
        if self.G_WGRAD_ON_D_STREAM is not None:
            return bool(self.G_WGRAD_ON_D_STREAM)
        env = os.environ.get("DCGAN_G_WGRAD_ON_D")
        if env in ("0", "1"):
            return env == "1"
        # 128x128 bf16 with the G weight gradients beside the chains (alt1): 34.4k-34.5k vs
        # 33.8k-33.9k img/s; 256x256 fp16 within the noise, kept on cs
        # (profiles/r5/ab_gw_place_128_256_r5.txt)
        return self.cfg.output_size <= 128

    def _schedule(self) -> str:
        req = self._sched_req
        if self._timing:  # phase timers need the segmented step
            return req if req in ("concurrent", "serial") else "concurrent"
        if self.ddp:
            if req in ("ddp", "concurrent", "serial"):
                return req
            # "concurrent" by default: inside ONE hipGraph the collectives do not overlap the
            # compute branches on ROCm (emulated ring collectives, 64x64: 1.39 ms vs 1.33 for
            # the segmented step; profiles/r3/ab_ddp_one_graph_r3.txt)
            env = os.environ.get("DCGAN_DDP_SCHEDULE") or "concurrent"
            if env not in DDP_SCHEDULES:  # "fused" here would issue no all-reduce at all
                raise ValueError("DCGAN_DDP_SCHEDULE=%r: expected one of %s" % (env, ", ".join(DDP_SCHEDULES)))
            return env
        return req or "fused"

    def _one_graph(self) -> bool:
        return self._schedule() in ("fused", "ddp")

    def _segments(self):
        """The step as a list of (name, runner, stream) segments: runner(ex, stream, sec) issues the
        segment onto `stream` (+ `sec`, its slot-1 stream; multi-stream segments fork the alt
        streams from `stream` and join them back before they end). runner.empty: nothing to run
        (fp16 keeps both Adams in the last segment)."""
        sch = self._schedule()
        A, B, C, W = self.progA, self.progB, self.progC, self.progW
        M = self.MAIN
        lin = self._lin_segment
        if sch in ("fused", "ddp"):
            run = (lambda ex, cs, sec: self._run_fused(ex, cs)) if sch == "fused" else \
                (lambda ex, cs, sec: self._run_ddp(ex, cs))
            run.empty = False
            return [("step", run, M)]
        if sch == "concurrent" and self._sharded():
            return [("fwd", lin([(A, 0, self._a_fwd)]), M), ("D_bwd_top", lin([(B, 0, self._b_split)]), self.ALT),
                    ("G_chain", lin([]), M), ("D_bwd_rest", lin([(B, self._b_split, -1)]), self.ALT),
                    ("G_tail", lin([]), M), ("update", lin([(C, 0, -1)]), M)]
        if sch == "serial":
            return [("fwd+G_bwd", lin([(A, 0, -1), (W, 0, -1)]), M), ("D_bwd_top", lin([(B, 0, self._b_split)]), M),
                    ("D_bwd_rest", lin([(B, self._b_split, -1)]), M), ("adam_G", lin([(C, 0, self._c_split)]), M),
                    ("adam_D", lin([(C, self._c_split, -1)]), M)]
        # "concurrent": one graph per chain segment, each on its own stream; the collectives go
        # out between them (ROCm refuses events recorded inside a graph that outside work waits
        # on: profiles/r2/probe_external_event_r2.txt). Graphs that fork and join both streams
        # around the collectives measured slower (profiles/r5/ab_ddp_5graph_joined_r5.txt).
        X = self.progX
        wx = lambda name: ([(X, self._wire_ops[name], self._wire_ops[name] + 1)]  # noqa: E731
                           if self._wire_direct() and name in self._wire_ops else [])
        sp = self._g_split
        if sp is None:
            g_chain, g_tail = [(A, self._a_fwd, -1), (W, 0, -1)] + wx("g"), []
        else:  # G's lowest deconv weight gradient ends the chain; the rest of G's backward follows
            a_need, wb, we = sp[:3]
            g_chain = [(A, self._a_fwd, a_need), (W, wb, we)] + wx("g_a")
            g_tail = [(A, a_need, -1), (W, 0, wb), (W, we, -1)] + wx("g_b") + wx("g_c")
        segs = [("fwd", lin([(A, 0, self._a_fwd)]), M),
                ("D_bwd_top", lin([(B, 0, self._b_split)] + wx("dtop")), self.ALT),
                ("G_chain", lin(g_chain), M),
                ("D_bwd_rest", lin([(B, self._b_split, -1)] + wx("drest")), self.ALT),
                ("G_tail", lin(g_tail), M)]
        if self._adam_g_split():
            segs.append(("adam_G_a", lin([(C, self._c_split, self._c_split_a)]), M))
        return segs + [("adam_D", lin([(C, 0, self._c_split)]), M),
                       ("adam_G", lin([(C, self._c_split_a, -1)]), M)]

    @staticmethod
    def _lin_segment(parts):
        def run(ex, cs, sec):
            for prog, b, e in parts:
                ex.run(prog, [cs, sec], b, e)
        run.empty = all((prog.size() if e < 0 else e) <= b for prog, b, e in parts)
        return run

    def _w_begin(self, k: int) -> int:
        return self._g_w[k - 1][1] if k > 0 else 0

    def enable_timing(self) -> None:
        """Per-phase GPU timers: the step runs as segments with events between
        them. Call before the first train_step (graphs are captured per segment). Concurrent
        schedule: each phase is reported as ms from the step start to the END of that phase
        (the D and G chains overlap); serial schedule: phase durations. The update program is
        rebuilt for the segmented schedule (Adam(G) and Adam(D) apart)."""
        if self._graphs or self._step_host:
            raise RuntimeError("enable_timing() must precede the first train_step")
        self._timing = True
        self._build_updates()
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

    def _tick(self, i, stream) -> None:
        if self._timing and not self.dry:
            self._ev[i].record(stream)

    def _get_exec(self):
        if self._exec is None:
            self._exec = _TorchExec(self)
        return self._exec

    def _run_fused(self, ex, cs):
        """The "fused" schedule issued onto cs (+ the alt streams); also what gets captured. D's
        backward starts right after the forward (profiles/r4/ab_d_start_after_r4.txt); G's weight
        gradients run on the streams _gw_place() gives."""
        ex.run(self.progA, [cs, ex.side], 0, self._a_fwd)
        ex.wait(ex.alt[0], cs)
        ex.run(self.progB, ex.alt)
        # the G chain: data gradients on cs; each G weight gradient on its _gw_place() stream once
        # cs has produced its operand (a mark after that progA position)
        if not self._g_wgrad_on_d_stream():  # every G gradient on cs
            ex.run(self.progA, [cs, ex.side], self._a_fwd, -1)
            ex.run(self.progW, [cs, ex.side])
            ex.wait(cs, ex.alt[0])
            ex.run(self.progC, [cs, ex.side])
            return
        pos, marks = self._a_fwd, []
        for a_end, _ in self._g_w:
            ex.run(self.progA, [cs, ex.side], pos, a_end)
            marks.append(ex.mark(cs))
            pos = a_end
        ex.run(self.progA, [cs, ex.side], pos, -1)
        place = self._gw_place()
        streams = {"d": ex.alt, "s": [ex.side], "a": [ex.alt[1]]}
        w, segs = 0, []
        for k, (m, (_, w_end)) in enumerate(zip(marks, self._g_w)):
            segs.append((place[k], w, w_end))
            if place[k] != "c":
                st = streams[place[k]]
                ex.wait_mark(st[0], m)
                ex.run(self.progW, st, w, w_end)
            w = w_end
        for q in sorted(set(place) & {"s", "a"}):
            ex.wait(cs, streams[q][0])
        # the G weight gradients placed on cs run after the G chain (their operands are produced
        # there)
        for q, lo, hi in segs:
            if q == "c":
                ex.run(self.progW, [cs, ex.side], lo, hi)
        ex.wait(cs, ex.alt[0])
        ex.run(self.progC, [cs, ex.side])

    def _gw_place(self) -> str:
        """Stream of each G weight-gradient segment in the fused step: "a" (default) the idle alt1
        stream as soon as its operand exists, "s" the side stream, "d" behind the D chain, "c" on
        cs after the G chain; DCGAN_GW_PLACE gives one letter per segment ("aaaa" measured best,
        profiles/r5/ab_gw_place_r5.txt)."""
        n = len(self._g_w)
        v = os.environ.get("DCGAN_GW_PLACE")
        if v is None:
            return "a" * n
        if len(v) != n or set(v) - set("dcsa"):
            raise ValueError("DCGAN_GW_PLACE must be %d letters of d/c/s/a, got %r" % (n, v))
        return v

    def _seg(self, ex, i, stream):
        """Run segment i on `stream` (graph replay, or eager replay of its program ranges)."""
        if self.graph_enabled:
            g = self._graphs[i]
            if g is not None:
                ex.replay(g, stream)
            return
        _, run, which = self._segments()[i]
        run(ex, stream, ex.side if which == self.MAIN else ex.alt[1])

    def _run_step(self, ex):
        cs = ex.main()
        sch = self._schedule()
        if sch in ("fused", "ddp"):
            if self.graph_enabled:
                self._seg(ex, 0, cs)
            elif sch == "fused":
                self._run_fused(ex, cs)
            else:
                self._run_ddp(ex, cs)
            return
        self._run_segmented(ex, cs, sch)

    def _capture(self):
        """Capture the step: "fused" and "ddp" as ONE hipGraph ("ddp" with its RCCL collectives
        inside), the segmented schedules one graph per segment (their collectives stay outside,
        issued between replays on the comm stream). Capturing does not execute anything; it is
        attempted only after one eager step has loaded every code object, and any failure
        falls back to eager replay of the recorded programs."""
        ex = self._get_exec()
        sch = self._schedule()
        if sch == "ddp" and self.ddp and D.is_initialized() and D.backend() != "nccl":
            return False  # host-synchronous collectives (gloo) cannot be captured
        try:
            torch.cuda.synchronize(self.device)
            graphs = []
            one = self._one_graph()
            for name, run, which in self._segments():
                if run.empty:
                    graphs.append(None)  # empty segment (fp16: no separate G update)
                    continue
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    cs = torch.cuda.current_stream(self.device)
                    if one and self.ddp:
                        ex.wait(ex.comm, cs)  # the comm stream joins the capture from its start
                    run(ex, cs, ex.side if which == self.MAIN else ex.alt[1])
                graphs.append(g)
            self._graphs = graphs
            return True
        except Exception as e:  # pragma: no cover - depends on runtime
            print("[hip_engine] graph capture failed, running eagerly: %s" % e)
            self._graphs = []
            return False

    def train_step(self) -> None:
        if self.dry:
            raise RuntimeError("a dry-run engine only records the step (engine.schedule_check)")
        self._ensure_comm()
        if (self.graph_requested and not self.graph_enabled and self._step_host >= 1
                and not getattr(self, "_cap_tried", 0)):
            self._cap_tried = 1
            self.graph_enabled = self._capture()
        self._run_step(self._get_exec())
        self._step_host += 1
        # one EMA update per BN slot per step (zero-debias bookkeeping, host-side counters)
        self.model.g_bn.count_step(0)
        for s in range(self.model.d_bn.slots):
            self.model.d_bn.count_step(s)

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

    def sync_state_for_checkpoint(self) -> None:
        torch.cuda.synchronize(self.device)

    def sync_bn_state(self) -> None:
        """Average BN moving averages over ranks (collective; see ReferenceEngine) -- and, after
        sharded updates, gather the conv kernels' fp32 masters and Adam slots (checkpoints)."""
        self.gather_sharded_state()
        D.all_reduce_mean_(self.model.g_bn.flat)
        D.all_reduce_mean_(self.model.d_bn.flat)

    def after_state_load(self) -> None:
        """Call after loading weights/slots from a checkpoint: refresh the 16-bit weight mirrors."""
        self._repack_weights_now()
