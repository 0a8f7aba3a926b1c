"""DCGAN generator / discriminator / sampler over TF-named, TF-laid-out parameters.

Parameters of each network live in ONE flat fp32 buffer (``ParamSet.flat``); every TF
variable (``g_h1/w``, ``d_bn2/gamma``, ...) is a view into it with its TF shape and
layout. The flat buffer is what the fused HIP Adam updates, what the
RCCL all-reduce reduces and what the rank-0 broadcast sends; the named views are what
the checkpoint writes.

The forward functions here are the *reference* (oracle) implementation on top of
``ops.reference`` and are differentiable with autograd. They mirror
``/root/reference/distriubted_model.py:83-153``:

* ``generator``: linear -> reshape NHWC -> [BN -> ReLU -> deconv]* -> tanh
* ``discriminator``: conv -> lrelu -> [conv -> BN -> lrelu]* -> NHWC flatten -> linear
* ``sampler``: generator with BN in inference mode (moving averages)

The discriminator accepts a batch made of ``groups`` equal parts with independent BN
statistics, so D(real) and D(fake) can run as one 2B batch while keeping the
reference's separate per-call statistics (``image_train.py:82,85``).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from ..ops import reference as R
from .config import DCGANConfig


# --------------------------------------------------------------------------- init
def truncated_normal_(t: torch.Tensor, std: float, gen: torch.Generator) -> torch.Tensor:
    """TF truncated_normal_initializer: N(0, std) resampled outside +-2 std."""
    flat = t.view(-1)
    out = torch.empty(flat.numel(), dtype=torch.float32)
    filled = 0
    while filled < out.numel():
        cand = torch.randn(out.numel() - filled, generator=gen) * std
        keep = cand[cand.abs() <= 2 * std]
        out[filled:filled + keep.numel()] = keep
        filled += keep.numel()
    flat.copy_(out.to(flat.dtype))
    return t


def init_tensor_(t: torch.Tensor, kind: str, std: float, gen: torch.Generator) -> None:
    with torch.no_grad():
        if kind == "zeros":
            t.zero_()
        elif kind == "normal":
            t.copy_(torch.randn(t.shape, generator=gen) * std)
        elif kind == "truncated":
            truncated_normal_(t, std, gen)
        elif kind == "gamma":  # random_normal_initializer(1., 0.02)
            t.copy_(1.0 + torch.randn(t.shape, generator=gen) * std)
        else:
            raise ValueError(kind)


# --------------------------------------------------------------------------- storage
class ParamSet:
    """Named views over one flat fp32 buffer. Offsets are 64-element aligned so every
    tensor starts on a 256-byte boundary (vector loads in the HIP kernels)."""

    ALIGN = 64

    def __init__(self, specs: Sequence[Tuple[str, Tuple[int, ...], str]],
                 device: torch.device | str = "cpu", dtype: torch.dtype = torch.float32):
        self.specs = list(specs)
        self.offsets: "OrderedDict[str, Tuple[int, Tuple[int, ...]]]" = OrderedDict()
        # storage order: every tensor the step reads in fp32 (biases, BN scale / offset, linear
        # layers) first, then the conv / deconv kernels ("/w") in layer order -- the tensors the
        # GEMMs only read through the 16-bit mirror. Each layer's kernel is then one contiguous
        # slice (DDP collectives per layer; the sharded update shards exactly those). Names, TF
        # shapes and the initialisation order stay the spec order.
        order = sorted(range(len(self.specs)), key=lambda i: (self.specs[i][0].endswith("/w"), i))
        offs = {}
        off = 0
        for i in order:
            name, shape, _ = self.specs[i]
            offs[name] = off
            off += -(-math.prod(shape) // self.ALIGN) * self.ALIGN
        for name, shape, _ in self.specs:
            self.offsets[name] = (offs[name], tuple(shape))
        self.numel_padded = off
        self.flat = torch.zeros(off, device=device, dtype=dtype)
        self._build_views()

    def _build_views(self) -> None:
        self.tensors: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for name, (off, shape) in self.offsets.items():
            self.tensors[name] = self.flat[off:off + math.prod(shape)].view(shape)

    @property
    def numel(self) -> int:
        return sum(math.prod(s) for _, s, _ in self.specs)

    def __getitem__(self, name: str) -> torch.Tensor:
        return self.tensors[name]

    def names(self) -> List[str]:
        return list(self.tensors.keys())

    def like(self, dtype: Optional[torch.dtype] = None) -> "ParamSet":
        """A zero ParamSet with the same layout (grads, Adam slots)."""
        p = ParamSet.__new__(ParamSet)
        p.specs = self.specs
        p.offsets = self.offsets
        p.numel_padded = self.numel_padded
        p.flat = torch.zeros_like(self.flat, dtype=dtype or self.flat.dtype)
        p._build_views()
        return p

    def to(self, device) -> "ParamSet":
        p = ParamSet.__new__(ParamSet)
        p.specs = self.specs
        p.offsets = self.offsets
        p.numel_padded = self.numel_padded
        p.flat = self.flat.to(device)
        p._build_views()
        return p

    def initialize(self, gen: torch.Generator, std: float = 0.02) -> None:
        for name, _, kind in self.specs:
            init_tensor_(self.tensors[name], kind, std, gen)

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        return OrderedDict((k, v.detach().cpu().clone()) for k, v in self.tensors.items())

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> List[str]:
        missing = []
        with torch.no_grad():
            for k, v in self.tensors.items():
                if k in sd:
                    src = torch.as_tensor(sd[k])
                    if tuple(src.shape) != tuple(v.shape):
                        raise ValueError("shape mismatch for %s: %s vs %s" % (k, tuple(src.shape), tuple(v.shape)))
                    v.copy_(src.to(v.dtype))
                else:
                    missing.append(k)
        if strict and missing:
            raise KeyError("missing variables: %s" % missing)
        return missing


class BNState:
    """BN moving averages (reference ``batch_norm`` EMA, ``distriubted_model.py:23,41``).

    G BN layers have one (mean, var) shadow pair each; D BN layers have one pair per
    D call in the reference step (real, fake) -> ``slots = 2``. Shadows start at zero
    (TF slot initialiser for tensor inputs). With ``zero_debias`` the TF>=0.12 form is
    used (biased accumulator / (1 - decay^t)).
    """

    def __init__(self, layers: Sequence[Tuple[str, int]], slots: int, device="cpu",
                 decay: float = 0.9, zero_debias: bool = False):
        self.layers = list(layers)
        self.slots = slots
        self.decay = decay
        self.zero_debias = zero_debias
        total = sum(2 * slots * c for _, c in self.layers)
        self.flat = torch.zeros(total, device=device, dtype=torch.float32)
        self.steps = torch.zeros(slots, dtype=torch.float64)  # host-side debias counters
        self.mean: Dict[str, torch.Tensor] = {}
        self.var: Dict[str, torch.Tensor] = {}
        off = 0
        for name, c in self.layers:
            self.mean[name] = self.flat[off:off + slots * c].view(slots, c)
            off += slots * c
            self.var[name] = self.flat[off:off + slots * c].view(slots, c)
            off += slots * c

    @torch.no_grad()
    def update(self, name: str, slot: int, batch_mean: torch.Tensor, batch_var: torch.Tensor) -> None:
        a = 1.0 - self.decay
        self.mean[name][slot].sub_(a * (self.mean[name][slot] - batch_mean.detach().float()))
        self.var[name][slot].sub_(a * (self.var[name][slot] - batch_var.detach().float()))

    def count_step(self, slot: int) -> None:
        self.steps[slot] += 1

    def averages(self, name: str, slot: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        m, v = self.mean[name][slot], self.var[name][slot]
        if self.zero_debias:
            t = float(self.steps[slot])
            if t > 0:
                corr = 1.0 - self.decay ** t
                return m / corr, v / corr
        return m, v

    def tf_names(self, prefix_by_slot: Optional[Sequence[str]] = None) -> "OrderedDict[str, torch.Tensor]":
        """TF checkpoint keys of the shadow variables (TF>=0.12 ``tf.nn.moments`` naming:
        ``<scope>/moments/Squeeze[_1]/ExponentialMovingAverage``; the second call of a
        BN scope in the reference graph gets the ``<scope>_1`` name scope)."""
        out = OrderedDict()
        for name, _ in self.layers:
            for s in range(self.slots):
                scope = name if s == 0 else "%s_%d" % (name, s)
                out["%s/moments/Squeeze/ExponentialMovingAverage" % scope] = self.mean[name][s]
                out["%s/moments/Squeeze_1/ExponentialMovingAverage" % scope] = self.var[name][s]
        return out


# --------------------------------------------------------------------------- model
class DCGAN:
    """Parameters + BN state of one DCGAN; reference forward functions."""

    def __init__(self, cfg: DCGANConfig, device="cpu", seed: int = 0, zero_debias: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.g = ParamSet(cfg.g_variables(), device=self.device)
        self.d = ParamSet(cfg.d_variables(), device=self.device)
        gen = torch.Generator().manual_seed(int(seed))
        # init on CPU with a CPU generator, then copy (deterministic across devices)
        gi = ParamSet(cfg.g_variables())
        gi.initialize(gen, cfg.init_stddev)
        di = ParamSet(cfg.d_variables())
        di.initialize(gen, cfg.init_stddev)
        self.g.flat.copy_(gi.flat)
        self.d.flat.copy_(di.flat)
        self.g_bn = BNState(cfg.g_bn_layers(), slots=1, device=self.device,
                            decay=cfg.bn_momentum, zero_debias=zero_debias)
        self.d_bn = BNState(cfg.d_bn_layers(), slots=2, device=self.device,
                            decay=cfg.bn_momentum, zero_debias=zero_debias)

    # ---------------------------------------------------------------- reference G
    def generator(self, z: torch.Tensor, train: bool = True, P: Optional[Dict[str, torch.Tensor]] = None,
                  update_ema: bool = True, record: Optional[Dict[str, torch.Tensor]] = None) -> torch.Tensor:
        cfg = self.cfg
        P = P if P is not None else self.g.tensors
        B = z.shape[0]
        h = z @ P["g_h0_lin/Matrix"] + P["g_h0_lin/bias"]
        h = h.view(B, cfg.g_base_hw, cfg.g_base_hw, cfg.g_base_ch)
        h = self._bn(h, "g_bn0", P, self.g_bn, train, update_ema, groups=1, slots=(0,))
        h = torch.relu(h)
        if record is not None:
            record["g_h0"] = h
        for L in cfg.g_layers():
            h = R.conv2d_transpose_same(h, P[L.name + "/w"], (L.out_hw, L.out_hw), P[L.name + "/biases"])
            if record is not None:
                record[L.name + "/pre"] = h
            if L.bn:
                h = self._bn(h, L.bn, P, self.g_bn, train, update_ema, groups=1, slots=(0,))
                h = torch.relu(h)
            else:
                h = torch.tanh(h)
            if record is not None:
                record[L.name] = h
        return h

    def sampler(self, z: torch.Tensor) -> torch.Tensor:
        """Generator with BN in inference mode (``distriubted_model.py:131-153``)."""
        with torch.no_grad():
            return self.generator(z, train=False, update_ema=False)

    # ---------------------------------------------------------------- reference D
    def discriminator(self, x: torch.Tensor, groups: int = 1, slots: Sequence[int] = (0,),
                      train: bool = True, P: Optional[Dict[str, torch.Tensor]] = None,
                      update_ema: bool = True, record: Optional[Dict[str, torch.Tensor]] = None):
        """Returns (sigmoid(logits), logits) with logits [N,1] (``distriubted_model.py:114-128``)."""
        cfg = self.cfg
        P = P if P is not None else self.d.tensors
        h = x
        if record is not None:
            record["d_in"] = h
        for L in cfg.d_layers():
            h = R.conv2d_same(h, P[L.name + "/w"], P[L.name + "/biases"])
            if record is not None:
                record[L.name + "/pre"] = h
            if L.bn:
                h = self._bn(h, L.bn, P, self.d_bn, train, update_ema, groups=groups, slots=slots)
            h = R.lrelu(h, cfg.lrelu_leak)
            if record is not None:
                record[L.name] = h
        N = h.shape[0]
        logits = h.reshape(N, -1) @ P[cfg.d_lin_name + "/Matrix"] + P[cfg.d_lin_name + "/bias"]
        return torch.sigmoid(logits), logits

    # ---------------------------------------------------------------- BN
    def _bn(self, h, name, P, state: BNState, train, update_ema, groups, slots):
        beta, gamma = P[name + "/beta"], P[name + "/gamma"]
        if train:
            mean, var = R.moments(h, groups)
            if update_ema:
                for g, s in zip(range(groups), slots):
                    state.update(name, s, mean[g], var[g])
            return R.batch_norm(h, mean, var, beta, gamma, self.cfg.bn_eps, groups=groups)
        m, v = state.averages(name, slots[0])
        return R.batch_norm(h, m, v, beta, gamma, self.cfg.bn_eps)

    # ---------------------------------------------------------------- misc
    def all_named_variables(self) -> "OrderedDict[str, torch.Tensor]":
        out = OrderedDict()
        out.update(self.g.tensors)
        out.update(self.d.tensors)
        return out
