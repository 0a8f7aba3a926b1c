"""TF-exact reference ops in plain PyTorch (NHWC, any device, any float dtype).

These are the semantics contract and the oracle every HIP kernel
is tested against. They reproduce, with explicit padding/cropping:

* ``tf.nn.conv2d(..., padding='SAME')`` with HWIO weights (``distriubted_model.py:183``):
  asymmetric TF padding (pad_lo, pad_hi) -- *not* PyTorch's symmetric ``padding=2``.
* ``tf.nn.conv2d_transpose`` with ``[kh, kw, out, in]`` weights (``:200-201``): the exact
  adjoint of the SAME conv = full transposed conv cropped to ``[pad_lo : pad_lo + out]``.
* ``batch_norm_with_global_normalization`` with biased batch moments over N,H,W (``:37,49``).
* ``lrelu`` = max(x, leak*x) (``:157``), ``sigmoid_cross_entropy_with_logits``
  (``image_train.py:91-95``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ..models.config import same_pads


def conv2d_same(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
                stride: int = 2) -> torch.Tensor:
    """x: [B,H,W,Cin] NHWC, w: [kh,kw,Cin,Cout] (HWIO) -> [B,ceil(H/s),ceil(W/s),Cout]."""
    kh, kw = w.shape[0], w.shape[1]
    ph = same_pads(x.shape[1], kh, stride)
    pw = same_pads(x.shape[2], kw, stride)
    xn = x.permute(0, 3, 1, 2)
    xn = F.pad(xn, (pw[0], pw[1], ph[0], ph[1]))
    y = F.conv2d(xn, w.permute(3, 2, 0, 1), None, stride=stride)
    y = y.permute(0, 2, 3, 1)
    if b is not None:
        y = y + b
    return y


def conv2d_transpose_same(x: torch.Tensor, w: torch.Tensor, out_hw: Tuple[int, int],
                          b: Optional[torch.Tensor] = None, stride: int = 2) -> torch.Tensor:
    """x: [B,Hi,Wi,Cin], w: [kh,kw,Cout,Cin] -> [B,Ho,Wo,Cout] (TF 'SAME' conv2d_transpose)."""
    kh, kw = w.shape[0], w.shape[1]
    ho, wo = out_hw
    ph = same_pads(ho, kh, stride)
    pw = same_pads(wo, kw, stride)
    xn = x.permute(0, 3, 1, 2)
    full = F.conv_transpose2d(xn, w.permute(3, 2, 0, 1), None, stride=stride)
    y = full[:, :, ph[0]:ph[0] + ho, pw[0]:pw[0] + wo]
    y = y.permute(0, 2, 3, 1)
    if b is not None:
        y = y + b
    return y


def moments(x: torch.Tensor, groups: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-group, per-channel biased mean/variance over (N,H,W) (or (N) for 2-D x).

    ``groups`` splits the batch into equal contiguous groups with independent statistics
    (used to run D's real and fake passes as one 2B batch while keeping TF's separate
    per-call statistics). Returns [groups, C] tensors.
    """
    C = x.shape[-1]
    xg = x.reshape(groups, -1, C)
    mean = xg.mean(dim=1)
    var = (xg - mean[:, None, :]).pow(2).mean(dim=1)
    return mean, var


def batch_norm(x: torch.Tensor, mean: torch.Tensor, var: torch.Tensor, beta: torch.Tensor,
               gamma: torch.Tensor, eps: float = 1e-5, groups: int = 1) -> torch.Tensor:
    """TF batch_norm_with_global_normalization(scale_after_normalization=True).

    mean/var: [C] or [groups, C]."""
    if mean.dim() == 1:
        return (x - mean) * torch.rsqrt(var + eps) * gamma + beta
    shp = x.shape
    C = shp[-1]
    xg = x.reshape(groups, -1, C)
    y = (xg - mean[:, None, :]) * torch.rsqrt(var[:, None, :] + eps) * gamma + beta
    return y.reshape(shp)


def lrelu(x: torch.Tensor, leak: float = 0.2) -> torch.Tensor:
    return torch.maximum(x, leak * x)


def sigmoid_cross_entropy_with_logits(logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    """TF formula: max(x,0) - x*t + log(1 + exp(-|x|))."""
    return logits.clamp(min=0) - logits * targets + torch.log1p(torch.exp(-logits.abs()))


def gan_losses(d_logits_real: torch.Tensor, d_logits_fake: torch.Tensor):
    """(d_loss_real, d_loss_fake, g_loss, d_loss) exactly as image_train.py:91-96."""
    d_real = sigmoid_cross_entropy_with_logits(d_logits_real, torch.ones_like(d_logits_real)).mean()
    d_fake = sigmoid_cross_entropy_with_logits(d_logits_fake, torch.zeros_like(d_logits_fake)).mean()
    g = sigmoid_cross_entropy_with_logits(d_logits_fake, torch.ones_like(d_logits_fake)).mean()
    return d_real, d_fake, g, d_real + d_fake


def tf_adam_update(param: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                   beta1_power: float, beta2_power: float, lr: float, beta1: float,
                   beta2: float = 0.999, eps: float = 1e-8) -> None:
    """One TF ``ApplyAdam`` (in place). beta*_power are the values *before* this step's
    update, i.e. beta^t for the t-th step (TF keeps them as variables initialised to beta)."""
    lr_t = lr * (1.0 - beta2_power) ** 0.5 / (1.0 - beta1_power)
    m.mul_(beta1).add_(grad, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(grad, grad, value=1.0 - beta2)
    param.sub_(lr_t * m / (v.sqrt() + eps))


def zero_fraction(x: torch.Tensor) -> torch.Tensor:
    """tf.nn.zero_fraction (sparsity summary, distriubted_model.py:80)."""
    return (x == 0).float().mean()
