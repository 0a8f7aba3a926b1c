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

import math
import os
from typing import Dict, List, Optional, Tuple

import torch

from ..models.config import DCGANConfig, same_pads
from ..models.dcgan import DCGAN
from ..optim.adam import TFAdam
from ..ops import hip as H
from ..parallel import dist as D
from .hip_aux import HipEngineAux

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


class HipEngine(HipEngineAux):
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

    # ---- sharded update (segmented DDP step, bf16): reduce-scatter -> Adam on 1/W -> all-gather
    def _shard_plan(self):
        """(name, model, a, b) of the sharded slices -- the conv kernels, which the step reads only
        through the 16-bit mirror (ParamSet stores them last, in layer order) -- and the
        (name, model, a, b) all-reduced slices of everything it reads in fp32 (biases, BN
        scale / offset, linear layers), or None where the sharded update does not apply."""
        if not (self.ddp and self.dt == 0 and not self.graph_requested and self._g_split is not None
                and os.environ.get("DCGAN_DDP_SHARD", "1") != "0"):
            return None
        Dm, G = self.model.d, self.model.g
        first_w = lambda ps: min(off for k, (off, _) in ps.offsets.items() if k.endswith("/w"))  # noqa: E731
        sdw, o, nd = first_w(Dm), self._d_top_off, Dm.flat.numel()
        lo, hi = self._g_split[3:]
        W = self.shard_world or self.world
        if lo != first_w(G) or not (sdw < o < nd) or any((b - a) % W for a, b in ((sdw, o), (o, nd), (lo, hi))):
            return None
        shard = [("dw_top", "d", o, nd), ("g_b", "g", hi, G.flat.numel()), ("g_a", "g", lo, hi), ("dw_rest", "d", sdw, o)]
        return shard, [("d_small", "d", 0, sdw), ("g_c", "g", 0, lo)]

    shard_world: Optional[int] = None  # shard count override (the one-GPU RCCL-like stand-in)

    def _sharded(self) -> bool:
        return getattr(self, "_shards", None) is not None and self._schedule() == "concurrent"

    def _build_shards(self):
        """ShardReducers (their reduced-gradient / 16-bit shard buffers) and progSh: one Adam per
        shard, run on the comm stream between its reduce-scatter and its all-gather."""
        plan = self._shard_plan()
        self._shards, self._sh_ops, self.progSh = None, {}, None
        if plan is None:
            return
        W = self.shard_world or self.world
        r = self.rank % W
        self._shards, self._small = {}, plan[1]
        self.progSh = self._prog()
        for name, m, a, b in plan[0]:
            ps, grad, mir = ((self.model.d, self.grad_d, self.wbf_d) if m == "d" else (self.model.g, self.grad_g, self.wbf_g))
            opt = self.opt_d if m == "d" else self.opt_g
            sr = D.ShardReducer(grad.flat[a:b], mir.flat[a:b], W, r)
            self._shards[name] = (sr, m, a, b)
            k = a + sr.lo
            i0 = self.progSh.size()
            self.progSh.adam_bf("adam_shard." + name, _p(ps.flat) + 4 * k, _p(sr.agin), _p(sr.gs),
                                _p(opt.m.flat) + 4 * k, _p(opt.v.flat) + 4 * k, _p(opt.powers), sr.n, opt.lr,
                                opt.beta1, opt.beta2, opt.eps, 1.0 / self.world, 0, 0, 0)
            self._sh_ops[name] = (i0, self.progSh.size())

    def _build_update_sharded(self, prog):
        """Adam over the all-reduced fp32-read slices (full, every rank) + both beta powers + the
        step counter, after every shard's Adam has read the powers (the step's final join)."""
        gs = 1.0 / self.world
        for name, m, a, b in self._small:
            ps, grad, mir, opt = ((self.model.d, self.grad_d, self.wbf_d, self.opt_d) if m == "d" else
                                  (self.model.g, self.grad_g, self.wbf_g, self.opt_g))
            es = mir.flat.element_size()
            prog.adam_bf("adam." + name, _p(ps.flat) + 4 * a, _p(mir.flat) + es * a, _p(grad.flat) + 4 * a,
                         _p(opt.m.flat) + 4 * a, _p(opt.v.flat) + 4 * a, _p(opt.powers), b - a, opt.lr, opt.beta1,
                         opt.beta2, opt.eps, gs, 0, 0, 0)
        od, og = self.opt_d, self.opt_g
        prog.step_end("step_end", _p(od.powers), _p(og.powers), od.beta1, od.beta2, og.beta1, og.beta2,
                      _p(self.step_counter), 0, 0, self.LOSS_SCALE_GROWTH)

    def _sh_rs(self, ex, name, src) -> None:
        if self.ddp:
            ex.wait(ex.comm, src)
            ex.collective(self._shards[name][0].rs_op, ex.comm)

    def _sh_update(self, ex, name) -> None:
        """Adam over this rank's shard (on the comm stream, after its reduce-scatter), then the
        all-gather of the 16-bit shards into the mirror slice."""
        if self.ddp:
            b, e = self._sh_ops[name]
            ex.run(self.progSh, [ex.comm], b, e)
            ex.collective(self._shards[name][0].ag_op, ex.comm)

    def _run_sharded(self, ex, cs) -> None:
        """The segmented DDP step with the sharded update. Comm-stream order: RS(d_h3) as soon as
        D's top layer is done; Adam + AG of it once the g_loss pass has left D (mark inside the G
        chain); RS(g_h2..g_h4 kernels) from alt1; RS(g_h1 kernel) after the G chain, Adam + AG of
        g_h2..g_h4 (their last reader, the G chain, is done); RS / Adam / AG of D's lower kernels
        and the all-reduce of D's fp32-read tensors after the D chain; the all-reduce of G's after
        the G tail, then Adam + AG of g_h1 (its data gradient, in the tail, read the old mirror).
        The main stream joins the comm stream and runs Adam over the all-reduced slices."""
        alt = ex.alt[0]
        self._tick(0, cs)
        self._seg(ex, 0, cs)                   # z, G fwd, D fwd (real | fake), losses
        self._tick(1, cs)
        ex.wait(alt, cs)
        self._seg(ex, 1, alt)                  # D chain: head + top layer gradients
        self._tick(2, alt)
        self._sh_rs(ex, "dw_top", alt)
        gd = []                                # mark: the g_loss pass is done with D's weights
        self._g_chain_gw_alt(ex, cs, on_gd=gd.append, sharded=True)
        self._tick(3, cs)
        self._sh_rs(ex, "g_a", cs)
        self._sh_update(ex, "g_b")
        B, bt = self.progB, self._b_top_dgrad
        ex.run(B, ex.alt, self._b_split, bt)   # D chain: the top layer's data gradient
        if self.ddp:                           # Adam + AG of the top kernel after its last readers
            ex.wait_mark(ex.comm, gd[0])
            ex.wait(ex.comm, alt)
        self._sh_update(ex, "dw_top")
        ex.run(B, ex.alt, bt, -1)              # D chain: the rest -> grad_d final
        self._tick(4, alt)
        self._sh_rs(ex, "dw_rest", alt)
        self._sh_update(ex, "dw_rest")
        self._ar_launch(ex, "d_small", alt)
        self._g_tail_gw_alt(ex, cs)
        self._tick(5, cs)
        self._ar_launch(ex, "g_c", cs)
        self._sh_update(ex, "g_a")
        self._ar_join(ex, cs)
        ex.wait(cs, alt)                       # (W = 1 timing: the D chain itself)
        self._seg(ex, 5, cs)                   # Adam over the all-reduced slices, powers, step
        self._tick(6, cs)

    def sync_check_tensors(self):
        """What the cross-rank divergence check compares: the fp32 masters, or -- after sharded
        updates, where each rank's conv-kernel masters are current only on its shard -- the 16-bit
        mirrors plus the masters of the all-reduced slices."""
        if self._shards is None or not self._sharded():
            return [self.model.g.flat, self.model.d.flat]
        out = [self.wbf_g.flat, self.wbf_d.flat]
        for name, m, a, b in self._small:
            out.append((self.model.d if m == "d" else self.model.g).flat[a:b])
        return out

    def gather_sharded_state(self) -> None:
        """Collective (every rank): after sharded updates each rank holds only its shard of the
        conv kernels' fp32 masters and Adam slots current; gather them (checkpoints, summaries
        of the masters, the divergence check)."""
        if self._shards is None or not self.ddp or self.dry:
            return
        torch.cuda.synchronize(self.device)
        for sr, m, a, b in self._shards.values():
            ps, opt = (self.model.d, self.opt_d) if m == "d" else (self.model.g, self.opt_g)
            for flat in (ps.flat, opt.m.flat, opt.v.flat):
                D.gather_shards(flat, [(a, b)])

    def _build_update_d_first(self, prog):
        """Adam(D) (progC[:_c_split]), then Adam(G) + beta powers / global step: the step counter
        update must follow both Adams (each reads its model's beta powers)."""
        gs = 1.0 / self.world
        od, og = self.opt_d, self.opt_g
        ls = _p(self.loss_scale)
        mg = 0 if self.f32 else _p(self.wbf_g.flat)
        md = 0 if self.f32 else _p(self.wbf_d.flat)
        wd, wg = (_p(self.wire_d.flat), _p(self.wire_g.flat)) if self._wire_direct() else (0, 0)
        prog.adam_bf("adam_d", _p(self.model.d.flat), md, _p(self.grad_d.flat), _p(od.m.flat), _p(od.v.flat),
                     _p(od.powers), self.model.d.flat.numel(), od.lr, od.beta1, od.beta2, od.eps, gs, 0, ls, wd)
        self._c_split = prog.size()
        G = self.model.g
        es = 0 if self.f32 else self.wbf_g.flat.element_size()

        def adam_g(name, a, b):  # Adam(G) over G's flat range [a, b)
            if b > a:
                prog.adam_bf(name, _p(G.flat) + 4 * a, mg + es * a if mg else 0, _p(self.grad_g.flat) + 4 * a,
                             _p(og.m.flat) + 4 * a, _p(og.v.flat) + 4 * a, _p(og.powers), b - a, og.lr, og.beta1,
                             og.beta2, og.eps, gs, 0, ls, wg + 2 * a if wg else 0)
        n = G.flat.numel()
        if self._adam_g_split():
            lo, hi = self._g_split[3:]
            adam_g("adam_g_a", lo, hi)      # g_h1's slice: right after its own collective
            self._c_split_a = prog.size()
            adam_g("adam_g_b", hi, n)
            adam_g("adam_g_c", 0, lo)
        else:
            self._c_split_a = self._c_split
            adam_g("adam_g", 0, n)
        prog.step_end("step_end", _p(od.powers), _p(og.powers), od.beta1, od.beta2, og.beta1, og.beta2,
                      _p(self.step_counter), 0, ls, self.LOSS_SCALE_GROWTH)

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

    def _g_bucket_cuts(self) -> List[Tuple[int, int, int]]:
        """G's gradient buckets for the "ddp" schedule: (progW piece index, lo, hi) -- after G's
        weight-gradient piece k the flat slice [lo, hi) is final (that layer's weights, biases and
        BN parameters, whose BN backward precedes the piece's mark, plus every later layer's);
        a last bucket [0, lo) (projection + g_bn0, written at the end of progA) follows the join.
        Default: cut after the two lowest G deconvs (the largest weight tensors; at 64x64: 4.1 MB
        after g_h2, 13.1 MB after g_h1, 3.3 MB last). DCGAN_G_CUTS=g_h2,g_h1 names them."""
        env = os.environ.get("DCGAN_G_CUTS")
        names = ([s for s in env.split(",") if s] if env is not None else
                 [L.name for L in self.gl[:-1][:2]])
        offs = self.model.g.offsets
        cuts, hi = [], self.model.g.flat.numel()
        for k, layer in enumerate(self._g_w_layer):
            if layer in names:
                lo = offs[layer + "/w"][0]
                cuts.append((k, lo, hi))
                hi = lo
        cuts.append((len(self._g_w_layer), 0, hi))
        return cuts

    def _g_split_plan(self):
        """Where the segmented ("concurrent") DDP schedule splits G's gradient all-reduce: G's
        lowest deconv (g_h1 at 64x64: 13.1 of G's 20.5 MB) has its weight gradient computed as
        soon as its input gradient exists -- progA up to the position that piece needs, then the
        piece itself -- and its slice [lo, hi) (weights, bias, BN parameters) goes on the wire
        while the rest of G's backward (the g_h1 data gradient, g_bn0, the projection and the
        other layers' weight gradients) runs. Returns (a_need, w_begin, w_end, lo, hi) or None
        (one G all-reduce after the chain)."""
        if len(self.gl) < 2 or self.gl[0].name not in self._g_w_layer:
            return None
        k = self._g_w_layer.index(self.gl[0].name)
        a_need, w_end = self._g_w[k]
        w_begin = self._g_w[k - 1][1] if k > 0 else 0
        if w_end <= w_begin or a_need <= self._a_fwd:
            return None
        offs = self.model.g.offsets
        lo, hi = offs[self.gl[0].name + "/w"][0], offs[self.gl[1].name + "/w"][0]
        return a_need, w_begin, w_end, lo, hi

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

    def _adam_g_split(self) -> bool:
        """Segmented DDP step: Adam over g_h1's slice as soon as its collective has landed, Adam over
        the rest of G after the last one (DCGAN_ADAM_G_SPLIT=0: one Adam(G) at the end;
        profiles/r5/ab_adam_g_split_r5.txt)."""
        return (self._schedule() == "concurrent" and self._g_split is not None and not self.f16
                and os.environ.get("DCGAN_ADAM_G_SPLIT", "1") != "0")

    def _wire_direct(self) -> bool:
        """bf16 wire without copies (segmented DDP step, bf16 engine): cast kernels inside the
        step graphs write each gradient slice's bf16 image when the slice is final, RCCL reduces
        the image in place, Adam reads it (``adam_bf(gbf=...)``). Other schedules / dtypes use the
        reducer's own fp32 <-> bf16 copies around each collective."""
        return (self.wire_d is not None and self._schedule() == "concurrent" and not self._sharded()
                and os.environ.get("DCGAN_WIRE_DIRECT", "1") != "0")  # =0: the copying reducer (A/B)

    def _wire_cast(self, ex, name: str, streams) -> None:
        if self._wire_direct() and name in self._wire_ops:
            i = self._wire_ops[name]
            ex.run(self.progX, streams, i, i + 1)

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

    def _run_ddp(self, ex, cs):
        """The "ddp" schedule: the fused step with the gradient all-reduces on the comm stream,
        issued from inside the step (and captured with it into ONE hipGraph under RCCL).
        Comm-stream order = issue order: D's top layer + head (final after progB[:_b_split]),
        the rest of D's (the D chain ends first), G's buckets as G's weight gradients land
        (``_g_cuts``), G's last bucket once both chains have joined. Adam(D) waits for D's
        collectives only and runs under G's last one; Adam(G) + the step counter follow it."""
        alt = ex.alt[0]
        ex.run(self.progA, [cs, ex.side], 0, self._a_fwd)
        ex.wait(alt, cs)
        ex.run(self.progB, ex.alt, 0, self._b_split)
        self._ar_launch(ex, "dtop", alt)
        ex.run(self.progB, ex.alt, self._b_split, -1)
        self._ar_launch(ex, "drest", alt)
        d_done = ex.mark(ex.comm) if self.ddp else None
        cuts = {k: r for (k, _, _), r in zip(self._g_cuts[:-1], self._ar_gparts[:-1])}
        gw = self._g_wgrad_on_d_stream()
        pos, marks = self._a_fwd, []
        for a_end, _ in self._g_w:
            ex.run(self.progA, [cs, ex.side], pos, a_end)
            marks.append(ex.mark(cs))
            pos = a_end
        ex.run(self.progA, [cs, ex.side], pos, -1)
        wst = alt if gw else cs  # G weight gradients behind the D chain (64x64) or on cs
        w = 0
        for k, (m, (_, w_end)) in enumerate(zip(marks, self._g_w)):
            if gw:
                ex.wait_mark(alt, m)
            ex.run(self.progW, ex.alt if gw else [cs, ex.side], w, w_end)
            w = w_end
            if k in cuts and self.ddp:
                ex.wait(ex.comm, wst)
                ex.collective(cuts[k], ex.comm)
        ex.wait(cs, alt)
        if self.ddp:
            ex.wait(ex.comm, cs)
            ex.collective(self._ar_gparts[-1], ex.comm)
            ex.wait_mark(cs, d_done)
        ex.run(self.progC, [cs, ex.side], 0, self._c_split)   # Adam(D) under G's last bucket
        self._ar_join(ex, cs)
        ex.run(self.progC, [cs, ex.side], self._c_split, -1)  # Adam(G), beta powers, step

    def _seg(self, ex, i, stream):
        """Run segment i on `stream` (graph replay, or eager replay of its program ranges)."""
        if self.graph_enabled:
            g = self._graphs[i]
            if g is not None:
                ex.replay(g, stream)
            return
        _, run, which = self._segments()[i]
        run(ex, stream, ex.side if which == self.MAIN else ex.alt[1])

    def _ddp_gw_alt(self) -> bool:
        """Segmented DDP step, eager replay: G's weight gradients other than g_h1's on the idle alt1
        stream as soon as their operands exist, G's slice above g_h1 reduced from there
        (profiles/r5/ab_ddp_gw_alt_b_r5.txt, ab_ddp_gw_world_r5.txt)."""
        return (self._schedule() == "concurrent" and not (self.graph_enabled or self.graph_requested)
                and self._g_split is not None)

    def _g_chain_gw_alt(self, ex, cs, on_gd=None, sharded=False):
        """Segment "G_chain" with G's weight gradients on alt1 (_ddp_gw_alt), and the collective of
        G's slice above g_h1 as soon as they are done. on_gd(mark): called with a mark on cs once
        the g_loss pass is done with D's weights (progA[:_a_gd_end])."""
        A, W, a1 = self.progA, self.progW, ex.alt[1]
        a_need, wb, we = self._g_split[:3]
        pos, w = self._a_fwd, 0
        if on_gd is not None:
            ex.run(A, [cs, ex.side], pos, self._a_gd_end)
            on_gd(ex.mark(cs))
            pos = self._a_gd_end
        for a_end, w_end in self._g_w:
            if w_end > wb:
                break
            ex.run(A, [cs, ex.side], pos, a_end)
            ex.wait(a1, cs)
            ex.run(W, [a1], w, w_end)
            pos, w = a_end, w_end
        assert w == wb
        # G's slice above g_h1 (g_h2's weights on: "gsplit_b") is final once these weight
        # gradients are: its collective goes out now, into the comm stream's idle gap after D's top
        # layer, instead of after the G chain
        if sharded:
            self._sh_rs(ex, "g_b", a1)
        else:
            self._wire_cast(ex, "g_b", [a1])
            self._ar_launch(ex, "gsplit_b", a1)
        ex.run(A, [cs, ex.side], pos, a_need)
        ex.run(W, [cs, ex.side], wb, we)
        self._wire_cast(ex, "g_a", [cs, ex.side])

    def _g_tail_gw_alt(self, ex, cs) -> None:
        """Segment "G_tail" when G's weight gradients ran on alt1: the rest of the G chain, then
        the join with alt1 before G's remaining slices are cast / reduced."""
        we = self._g_split[2]
        ex.run(self.progA, [cs, ex.side], self._g_split[0], -1)
        ex.run(self.progW, [cs, ex.side], we, -1)
        ex.wait(cs, ex.alt[1])
        self._wire_cast(ex, "g_c", [cs, ex.side])

    def _ar_launch(self, ex, which: str, src) -> None:
        """All-reduce one gradient slice ("g", "dtop", "drest", "gsplit_a/b/c") on the comm stream
        once `src`'s queued work is done."""
        if self.ddp:
            r = getattr(self, "_ar_" + which)  # AttributeError: a collective _ensure_comm never built
            if r is None:                       # (an intentionally empty slice)
                return
            ex.wait(ex.comm, src)
            ex.collective(r, ex.comm)

    def _ar_join(self, ex, dst) -> None:
        """dst waits for every collective issued so far (the 1/W scale is folded into Adam)."""
        if self.ddp:
            ex.wait(dst, ex.comm)

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
        if sch == "concurrent" and self._sharded():
            self._run_sharded(ex, cs)
            return
        if sch == "concurrent":
            alt = ex.alt[0]
            self._tick(0, cs)
            self._seg(ex, 0, cs)               # z, G fwd, D fwd (real | fake), losses
            self._tick(1, cs)
            ex.wait(alt, cs)
            self._seg(ex, 1, alt)              # D chain: head + top layer gradients
            self._tick(2, alt)
            self._ar_launch(ex, "dtop", alt)
            gw = self._ddp_gw_alt()
            if gw:                             # the same segments with G's weight gradients on alt1
                self._g_chain_gw_alt(ex, cs)
            else:
                self._seg(ex, 2, cs)           # G chain: g_loss through D(fake), G backward to g_h1's wgrad
            self._tick(3, cs)
            a_done = None
            if self._g_split is not None:
                self._ar_launch(ex, "gsplit_a", cs)  # g_h1's slice, under the rest of both chains
                a_done = ex.mark(ex.comm) if self.ddp else None
            self._seg(ex, 3, alt)              # D chain: rest of D's backward -> grad_d final
            self._tick(4, alt)
            if gw:
                self._g_tail_gw_alt(ex, cs)
            else:
                self._seg(ex, 4, cs)           # G tail: g_h1 dgrad, g_bn0, projection, other G wgrads
            self._tick(5, cs)
            # D's last bucket, then the rest of G's; Adam(D) runs while G's is in flight
            self._ar_launch(ex, "drest", alt)
            d_done = ex.mark(ex.comm) if self.ddp else None
            if self._g_split is not None:
                if not gw:                     # (else issued from alt1 inside the G chain)
                    self._ar_launch(ex, "gsplit_b", cs)
                self._ar_launch(ex, "gsplit_c", cs)
            else:
                self._ar_launch(ex, "g", cs)
            i = 5
            if self._adam_g_split():
                if a_done is not None:
                    ex.wait_mark(cs, a_done)   # g_h1's collective (dtop's too: comm-stream order)
                self._seg(ex, i, cs)           # Adam over g_h1's slice, beside the other collectives
                i += 1
                self._tick(i, cs)
            if d_done is not None:
                ex.wait_mark(cs, d_done)       # dtop + drest (and g_h1's) collectives
            ex.wait(cs, alt)                   # (W = 1, timed: the D chain itself)
            self._seg(ex, i, cs)               # Adam D -> D mirror (overlaps G's all-reduce)
            self._tick(i + 1, cs)
            self._ar_join(ex, cs)              # G's collectives
            self._seg(ex, i + 1, cs)           # Adam G (the rest), step counter, G mirror
            self._tick(i + 2, cs)
            return
        self._tick(0, cs)
        self._seg(ex, 0, cs)                   # fwd, g_loss chain through D(fake), G backward -> grad_g final
        self._tick(1, cs)
        self._ar_launch(ex, "g", cs)
        g_done = ex.mark(ex.comm) if self.ddp else None
        self._seg(ex, 1, cs)                   # D backward: head + top layer (overlaps the G all-reduce)
        self._tick(2, cs)
        self._ar_launch(ex, "dtop", cs)
        self._seg(ex, 2, cs)                   # rest of D's backward -> grad_d final
        self._tick(3, cs)
        self._ar_launch(ex, "drest", cs)
        if g_done is not None:
            ex.wait_mark(cs, g_done)           # G's collective only
        self._seg(ex, 3, cs)                   # Adam G -> G mirror (overlaps the D all-reduces)
        self._tick(4, cs)
        self._ar_join(ex, cs)
        self._seg(ex, 4, cs)                   # Adam D, step counter, D mirror
        self._tick(5, cs)

    def _ensure_comm(self):
        """The gradient reducers of the current schedule (each owns its bf16 wire buffer when the
        wire is bf16, so only the ones the schedule issues are built)."""
        if self.ddp and not getattr(self, "_comm_built", False):
            self._comm_built = True
            o = self._d_top_off
            cs, mb, wd = self.comm_stream, self.bucket_mb, self.allreduce_dtype
            gf, df = self.grad_g.flat, self.grad_d.flat
            direct = self._wire_direct()
            wdf = self.wire_d.flat if direct else None
            wgf = self.wire_g.flat if direct else None

            # native RCCL only where the collectives are captured into the step's hipGraph ("ddp"):
            # issued eagerly, each ncclAllReduce cost ~50-60 us more than torch.distributed's
            # (profiles/r5/ab_native_rccl_eager_graph_r5.txt); captured, both cost the same
            native = (D.native_comm(self.device) if not self.dry and self._schedule() == "ddp" and self.graph_requested
                      else None)
            self.comm_kind = ("rccl-native" if native is not None else
                              "torch.distributed(%s)" % (D.backend() or "none"))

            def mk(t, wire=None):
                return D.GradAllReducer(t, mb, wd, stream=cs, force=True, wire=wire, prefilled=wire is not None,
                                        native=native)

            if self._sharded():  # the conv kernels go through ShardReducers; the fp32-read slices:
                for name, m, a, b in self._small:
                    setattr(self, "_ar_" + name, mk((df if m == "d" else gf)[a:b]) if b > a else None)
                return
            self._ar_dtop = mk(df[o:], wdf[o:] if direct else None)
            sch = self._schedule()
            self._ar_drest = mk(df[:o], wdf[:o] if direct else None)  # (also for graph-replayed segments)
            if sch == "serial" or (sch == "concurrent" and self._g_split is None):
                self._ar_g = mk(gf, wgf if direct else None)
            elif sch == "concurrent":  # g_h1's slice first, then the two others
                lo, hi = self._g_split[3:]
                self._ar_gsplit_a = mk(gf[lo:hi], wgf[lo:hi] if direct else None)
                self._ar_gsplit_b = mk(gf[hi:], wgf[hi:] if direct else None)
                self._ar_gsplit_c = mk(gf[:lo], wgf[:lo] if direct else None) if lo > 0 else None
            elif sch == "ddp":  # G's gradient in per-layer buckets (see _g_bucket_cuts)
                self._ar_gparts = [mk(gf[lo:hi]) for _, lo, hi in self._g_cuts]

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
