"""Reference (autograd) GAN training step -- the oracle for the fused HIP engine.

Semantics = ``image_train.py:151-158``: ONE forward of G,
D(real), D(fake) (separate BN statistics per D call), ``d_loss = d_real + d_fake``,
``g_loss`` non-saturating; D grads from ``d_loss`` w.r.t. ``d_`` vars, G grads from
``g_loss`` w.r.t. ``g_`` vars through D(fake) with *pre-update* D weights; both TF-Adam
updates applied in the same step; ``global_step`` incremented once (by G's optimiser).

Runs on any device (CPU for tests/plumbing, or GPU through PyTorch ops) and is also the
fallback engine when no HIP extension is available on CPU.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch

from ..models.dcgan import DCGAN
from ..ops import reference as R
from ..optim.adam import TFAdam


class ReferenceStep:
    def __init__(self, model: DCGAN, lr: float = 2e-4, beta1: float = 0.5,
                 grad_hook: Optional[Callable[[str, torch.Tensor], None]] = None):
        self.model = model
        self.opt_d = TFAdam(model.d, lr, beta1, power_suffix="")
        self.opt_g = TFAdam(model.g, lr, beta1, power_suffix="_1")
        self.global_step = 0
        self.grad_hook = grad_hook  # e.g. DDP all-reduce of the flat grad buffer
        self.last: Dict[str, torch.Tensor] = {}

    def forward_losses(self, real: torch.Tensor, z: torch.Tensor, Pg=None, Pd=None, update_ema=True,
                       record=None):
        m = self.model
        fake = m.generator(z, train=True, P=Pg, update_ema=update_ema, record=record)
        B = real.shape[0]
        both = torch.cat([real, fake], 0)
        _, logits = m.discriminator(both, groups=2, slots=(0, 1), train=True, P=Pd,
                                    update_ema=update_ema, record=record)
        lr_, lf = logits[:B], logits[B:]
        d_real, d_fake, g_loss, d_loss = R.gan_losses(lr_, lf)
        return {"fake": fake, "logits_real": lr_, "logits_fake": lf, "d_loss_real": d_real,
                "d_loss_fake": d_fake, "g_loss": g_loss, "d_loss": d_loss}

    def compute_grads(self, real: torch.Tensor, z: torch.Tensor, update_ema: bool = True):
        """Returns (losses dict, flat D grads, flat G grads) without applying them."""
        m = self.model
        Pg = {k: v.detach().clone().requires_grad_(True) for k, v in m.g.tensors.items()}
        Pd = {k: v.detach().clone().requires_grad_(True) for k, v in m.d.tensors.items()}
        out = self.forward_losses(real, z, Pg, Pd, update_ema=update_ema)
        d_names, g_names = m.d.names(), m.g.names()
        dg = torch.autograd.grad(out["d_loss"], [Pd[n] for n in d_names], retain_graph=True,
                                 allow_unused=True)
        gg = torch.autograd.grad(out["g_loss"], [Pg[n] for n in g_names], allow_unused=True)
        gd_flat = m.d.like()
        gg_flat = m.g.like()
        for n, g in zip(d_names, dg):
            if g is not None:
                gd_flat[n].copy_(g)
        for n, g in zip(g_names, gg):
            if g is not None:
                gg_flat[n].copy_(g)
        return out, gd_flat.flat, gg_flat.flat

    def step(self, real: torch.Tensor, z: torch.Tensor) -> Dict[str, float]:
        out, gd, gg = self.compute_grads(real, z)
        for s in range(2):  # one EMA update per BN slot per step (as the HIP engine counts)
            self.model.d_bn.count_step(s)
        self.model.g_bn.count_step(0)
        if self.grad_hook is not None:
            self.grad_hook("d", gd)
            self.grad_hook("g", gg)
        self.opt_d.step(gd)
        self.opt_g.step(gg)
        self.global_step += 1
        self.last = out
        return {k: float(out[k].detach()) for k in ("d_loss_real", "d_loss_fake", "g_loss", "d_loss")}
