"""DCGAN architecture description, parametric in output size / channels / depth.

The reference hard-codes a 64x64x3 model with ``gf_dim = df_dim = 64``
(``/root/reference/distriubted_model.py:7-12``) and an ``int(s/2^k)`` size ladder
(``:85``) that only works for sizes divisible by 16. Here the ladder is TF-'SAME'
consistent (``ceil``), the depth is configurable, and every layer's shape, TF variable
name and TF weight layout is derived in one place.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Tuple


def same_out(size: int, stride: int = 2) -> int:
    """Output size of a TF 'SAME' conv: ceil(in / stride)."""
    return -(-size // stride)


def same_pads(in_size: int, k: int = 5, stride: int = 2) -> Tuple[int, int]:
    """TF 'SAME' (pad_lo, pad_hi) for one spatial dim."""
    out = same_out(in_size, stride)
    total = max((out - 1) * stride + k - in_size, 0)
    lo = total // 2
    return lo, total - lo


def default_depth(output_size: int) -> int:
    """Stride-2 stages: 4 up to 64 px (reference), log2(size)-2 above (128 -> 5, 256 -> 6)."""
    return max(4, int(round(math.log2(max(output_size, 1)))) - 2)


@dataclass(frozen=True)
class ConvSpec:
    name: str          # TF scope, e.g. 'd_h1_conv' / 'g_h2'
    kind: str          # 'conv' (D, HWIO weight) | 'deconv' (G, [kh,kw,out,in] weight)
    in_hw: int
    out_hw: int
    cin: int
    cout: int
    bn: str | None     # BN scope name after this layer, or None
    act: str           # 'lrelu' | 'relu' | 'tanh' | 'none' applied after (BN or bias)

    @property
    def weight_shape(self) -> Tuple[int, int, int, int]:
        if self.kind == "conv":
            return (5, 5, self.cin, self.cout)
        return (5, 5, self.cout, self.cin)

    @property
    def pads(self) -> Tuple[int, int]:
        # for a deconv the pads are those of the adjoint conv (out_hw -> in_hw)
        return same_pads(self.in_hw if self.kind == "conv" else self.out_hw)


@dataclass(frozen=True)
class DCGANConfig:
    output_size: int = 64
    c_dim: int = 3
    gf_dim: int = 64
    df_dim: int = 64
    z_dim: int = 100
    depth: int = 0          # 0 -> default_depth(output_size)
    max_channels: int = 0   # 0 -> no cap
    bn_eps: float = 1e-5
    bn_momentum: float = 0.9
    lrelu_leak: float = 0.2
    init_stddev: float = 0.02

    @property
    def n_stages(self) -> int:
        return self.depth if self.depth > 0 else default_depth(self.output_size)

    def sizes(self) -> List[int]:
        """[s, s/2, s/4, ...] (ceil ladder), length n_stages + 1."""
        out = [self.output_size]
        for _ in range(self.n_stages):
            out.append(same_out(out[-1]))
        return out

    def _ch(self, base: int, mult: int) -> int:
        c = base * mult
        return min(c, self.max_channels) if self.max_channels > 0 else c

    # ------------------------------------------------------------------ G
    @property
    def g_base_hw(self) -> int:
        return self.sizes()[-1]

    @property
    def g_base_ch(self) -> int:
        return self._ch(self.gf_dim, 2 ** (self.n_stages - 1))

    @property
    def g_lin_out(self) -> int:
        return self.g_base_hw * self.g_base_hw * self.g_base_ch

    def g_layers(self) -> List[ConvSpec]:
        n = self.n_stages
        sizes = self.sizes()  # sizes[n] = base
        layers = []
        cin = self.g_base_ch
        for i in range(1, n + 1):
            in_hw, out_hw = sizes[n - i + 1], sizes[n - i]
            last = i == n
            cout = self.c_dim if last else self._ch(self.gf_dim, 2 ** (n - 1 - i))
            layers.append(ConvSpec(
                name="g_h%d" % i, kind="deconv", in_hw=in_hw, out_hw=out_hw, cin=cin, cout=cout,
                bn=None if last else "g_bn%d" % i, act="tanh" if last else "relu"))
            cin = cout
        return layers

    # ------------------------------------------------------------------ D
    def d_layers(self) -> List[ConvSpec]:
        n = self.n_stages
        sizes = self.sizes()
        layers = []
        cin = self.c_dim
        for i in range(n):
            cout = self._ch(self.df_dim, 2 ** i)
            layers.append(ConvSpec(
                name="d_h%d_conv" % i, kind="conv", in_hw=sizes[i], out_hw=sizes[i + 1],
                cin=cin, cout=cout, bn=None if i == 0 else "d_bn%d" % i, act="lrelu"))
            cin = cout
        return layers

    @property
    def d_lin_in(self) -> int:
        last = self.d_layers()[-1]
        return last.out_hw * last.out_hw * last.cout

    @property
    def d_lin_name(self) -> str:
        return "d_h%d_lin" % (self.n_stages - 1)

    # ------------------------------------------------------------------ variables
    def g_variables(self) -> List[Tuple[str, Tuple[int, ...], str]]:
        """(TF name, TF shape, init) for every G trainable, in TF creation order."""
        v = [("g_h0_lin/Matrix", (self.z_dim, self.g_lin_out), "normal"),
             ("g_h0_lin/bias", (self.g_lin_out,), "zeros"),
             ("g_bn0/beta", (self.g_base_ch,), "zeros"),
             ("g_bn0/gamma", (self.g_base_ch,), "gamma")]
        for L in self.g_layers():
            v.append((L.name + "/w", L.weight_shape, "normal"))
            v.append((L.name + "/biases", (L.cout,), "zeros"))
            if L.bn:
                v.append((L.bn + "/beta", (L.cout,), "zeros"))
                v.append((L.bn + "/gamma", (L.cout,), "gamma"))
        return v

    def d_variables(self) -> List[Tuple[str, Tuple[int, ...], str]]:
        v = []
        for L in self.d_layers():
            v.append((L.name + "/w", L.weight_shape, "truncated"))
            v.append((L.name + "/biases", (L.cout,), "zeros"))
            if L.bn:
                v.append((L.bn + "/beta", (L.cout,), "zeros"))
                v.append((L.bn + "/gamma", (L.cout,), "gamma"))
        v.append((self.d_lin_name + "/Matrix", (self.d_lin_in, 1), "normal"))
        v.append((self.d_lin_name + "/bias", (1,), "zeros"))
        return v

    def g_bn_layers(self) -> List[Tuple[str, int]]:
        out = [("g_bn0", self.g_base_ch)]
        out += [(L.bn, L.cout) for L in self.g_layers() if L.bn]
        return out

    def d_bn_layers(self) -> List[Tuple[str, int]]:
        return [(L.bn, L.cout) for L in self.d_layers() if L.bn]

    def param_counts(self) -> Dict[str, int]:
        g = sum(math.prod(s) for _, s, _ in self.g_variables())
        d = sum(math.prod(s) for _, s, _ in self.d_variables())
        return {"g": g, "d": d, "total": g + d}

    def flops_per_image(self) -> float:
        """Training FLOP/image with the reference step semantics."""
        gf = 2.0 * self.z_dim * self.g_lin_out
        for L in self.g_layers():
            gf += 2.0 * L.in_hw * L.in_hw * L.cin * L.cout * 25
        df = 0.0
        d0 = 0.0
        for i, L in enumerate(self.d_layers()):
            f = 2.0 * L.out_hw * L.out_hw * L.cin * L.cout * 25
            df += f
            if i == 0:
                d0 = f
        df += 2.0 * self.d_lin_in
        # G fwd + 2 D fwd + D wgrad (real+fake) + D dgrad d_loss chain (real+fake, not L0)
        # + D dgrad g_loss chain (fake, incl. L0) + G wgrad + G dgrad (no dgrad into z)
        g_lin = 2.0 * self.z_dim * self.g_lin_out
        return gf + 2 * df + 2 * df + 2 * (df - d0) + df + gf + (gf - g_lin)


def config_from_flags(flags) -> DCGANConfig:
    return DCGANConfig(output_size=int(flags.output_size), c_dim=int(flags.c_dim),
                       gf_dim=int(flags.gf_dim), df_dim=int(flags.df_dim), z_dim=int(flags.z_dim),
                       depth=int(flags.depth), max_channels=int(flags.max_channels))
