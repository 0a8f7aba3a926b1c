"""Data-parallel schedules of the HIP engine (mixin of ``hip_engine.HipEngine``), SURVEY.md §2.5.

The reference trains asynchronously through a gRPC parameter server (``image_train.py:156-158``,
``distriubted_model.py:70``); here every rank runs the same step and the gradients are combined over
RCCL on a comm stream while both backward chains keep running:

  "concurrent"  the step cut into segments (forward, D chain top / rest, G chain / tail, update) with
                per-slice all-reduces issued between them (fp32, or a copy-free bf16 wire) and Adam
                after them. DCGAN_DDP_SHARD=1 (bf16 engine, eager replay): the SHARDED update
                (``_run_sharded``) -- the conv kernels' gradients are reduce-scattered, each rank
                runs Adam on its 1/W shard on the comm stream and the bf16 mirror is all-gathered
                (0.75x the all-reduce's wire bytes at fp32 gradient precision, 1/W of the Adam
                work); the tensors the step reads in fp32 (biases, BN, linear layers) are
                all-reduced. Bit-identical to the all-reduce step, but slower under the RCCL-like
                stand-in at W = 2 / 4 / 8 (1.37 vs 1.29 ms at W=8: twice the collectives, each with
                its fixed latency, and g_h1's all-gather must wait for the G tail, its last reader;
                profiles/r6/ab_ddp_shard_standin_r6.txt), hence opt-in.
  "ddp"         the fused schedule with the all-reduces inside ONE hipGraph (native RCCL)
  "serial"      forward + G chain, then the D chain (the G all-reduce under D's backward)
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch

from ..parallel import dist as D


def _p(t) -> int:
    return 0 if t is None else int(t.data_ptr())


class HipDDPMixin:
    shard_world: Optional[int] = None  # shard count override (the one-GPU RCCL-like stand-in)

    def _shard_plan(self):
        """(name, model, a, b) of the sharded slices -- the conv kernels, which the step reads only
        through the 16-bit mirror (ParamSet stores them last, in layer order) -- and the
        (name, model, a, b) all-reduced slices of everything it reads in fp32 (biases, BN
        scale / offset, linear layers), or None where the sharded update does not apply."""
        if not (self.ddp and self.dt == 0 and not self.graph_requested and self._g_split is not None
                and os.environ.get("DCGAN_DDP_SHARD", "0") == "1"):
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
            # g_h2..g_h4's slice with it when its collective precedes g_h1's on the comm stream
            # (issued from alt1 inside the G chain: _ddp_gw_alt); stand-in W=8 1.288-1.291 vs
            # 1.302-1.303 ms (profiles/r6/ab_ddp_adam_order_r6.txt)
            early_b = self._ddp_gw_alt()
            if not early_b:
                self._c_split_a = prog.size()
            adam_g("adam_g_b", hi, n)
            if early_b:                     # (only the projection's Adam waits for the last collective)
                self._c_split_a = prog.size()
            adam_g("adam_g_c", 0, lo)
        else:
            self._c_split_a = self._c_split
            adam_g("adam_g", 0, n)
        prog.step_end("step_end", _p(od.powers), _p(og.powers), od.beta1, od.beta2, og.beta1, og.beta2,
                      _p(self.step_counter), 0, ls, self.LOSS_SCALE_GROWTH)

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

    def _adam_g_split(self) -> bool:
        """Segmented DDP step: Adam over g_h1's slice as soon as its collective has landed, Adam over
        the rest of G after the last one (DCGAN_ADAM_G_SPLIT=0: one Adam(G) at the end;
        profiles/r5/ab_adam_g_split_r5.txt)."""
        return (self._schedule() == "concurrent" and self._g_split is not None and not self.f16
                and os.environ.get("DCGAN_ADAM_G_SPLIT", "1") != "0")

    def _adam_d_alt(self) -> bool:
        """Segmented all-reduce DDP step, eager replay: Adam(D) on the D chain's stream as soon as
        D's collectives have landed, beside the G tail, instead of on the main stream after it
        (DCGAN_DDP_ADAM_D_ALT=0: after it). --force_ddp (W=1) 124.6-125.3k vs 122.2-122.4k img/s;
        stand-in W=2/4/8 within +-0.6 % (profiles/r6/ab_ddp_adam_order_r6.txt)."""
        return (self._ddp_gw_alt() and not self._sharded()
                and os.environ.get("DCGAN_DDP_ADAM_D_ALT", "1") != "0")

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

    def _run_segmented(self, ex, cs, sch):
        """The segmented DDP schedules ("concurrent", "serial"; also the per-phase timed step):
        graph segments or program ranges on the chain streams, collectives issued between them."""
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
            gd = []                            # mark: the g_loss pass is done with D's parameters
            if gw:                             # the same segments with G's weight gradients on alt1
                self._g_chain_gw_alt(ex, cs, on_gd=gd.append if self._adam_d_alt() else None)
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
            i = 6 if self._adam_g_split() else 5  # the "adam_D" segment
            d_alt = self._adam_d_alt()
            if d_alt:                          # Adam(D) on the D chain's stream once D's collectives
                if d_done is not None:         # have landed and the g_loss pass has left D, beside
                    ex.wait_mark(alt, d_done)  # the G tail
                ex.wait_mark(alt, gd[0])
                self._segments()[i][1](ex, alt, ex.alt[1])
                self._tick(i + 1, alt)
            if self._g_split is not None:
                if not gw:                     # (else issued from alt1 inside the G chain)
                    self._ar_launch(ex, "gsplit_b", cs)
                self._ar_launch(ex, "gsplit_c", cs)
            else:
                self._ar_launch(ex, "g", cs)
            if self._adam_g_split():
                if a_done is not None:
                    ex.wait_mark(cs, a_done)   # g_h1's collective (dtop's too: comm-stream order)
                self._seg(ex, 5, cs)           # Adam over g_h1's slice, beside the other collectives
                self._tick(6, cs)
            if d_alt:
                ex.wait(cs, alt)               # Adam(D) (before the step counter / beta powers)
            else:
                if d_done is not None:
                    ex.wait_mark(cs, d_done)   # dtop + drest (and g_h1's) collectives
                ex.wait(cs, alt)               # (W = 1, timed: the D chain itself)
                self._seg(ex, i, cs)           # Adam D -> D mirror (overlaps G's all-reduce)
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
