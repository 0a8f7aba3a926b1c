"""TF-form Adam over a flat parameter buffer (reference ``image_train.py:109-112``).

TF ``ApplyAdam``: ``lr_t = lr*sqrt(1-beta2^t)/(1-beta1^t)``, ``m = b1*m + (1-b1)*g``,
``v = b2*v + (1-b2)*g^2``, ``w -= lr_t*m/(sqrt(v)+eps)`` (eps *outside* the bias
correction, unlike torch.optim.Adam). Each optimiser keeps its own beta powers
(``beta1_power``/``beta2_power`` for D, ``beta1_power_1``/``beta2_power_1`` for G), which
are checkpointed -- the reference does not save them; we do, under TF's
slot names, so resume is exact.

On a GPU the update runs as ONE fused HIP kernel over the whole flat buffer
(``ops.hip.adam_``); the beta powers live on the device so the update can be captured in
a hipGraph. On CPU the reference formula runs.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Optional

import torch

from ..models.dcgan import ParamSet
from ..ops import reference as R


class TFAdam:
    def __init__(self, params: ParamSet, lr: float = 2e-4, beta1: float = 0.5, beta2: float = 0.999,
                 eps: float = 1e-8, power_suffix: str = ""):
        self.params = params
        self.lr, self.beta1, self.beta2, self.eps = float(lr), float(beta1), float(beta2), float(eps)
        self.m = params.like()
        self.v = params.like()
        dev = params.flat.device
        # [beta1_power, beta2_power] as TF variables (initialised to beta1, beta2), fp32
        self.powers = torch.tensor([self.beta1, self.beta2], dtype=torch.float32, device=dev)
        self.power_suffix = power_suffix
        self.use_hip = False

    @property
    def step_count(self) -> int:
        import math
        b1p = float(self.powers[0])
        return int(round(math.log(b1p) / math.log(self.beta1))) - 1 if b1p > 0 else 0

    def step(self, grads: torch.Tensor) -> None:
        """Apply one update from a flat grad buffer (same layout as params.flat)."""
        if self.use_hip:
            from ..ops import hip
            hip.adam_(self.params.flat, grads, self.m.flat, self.v.flat, self.powers,
                      self.lr, self.beta1, self.beta2, self.eps)
            return
        with torch.no_grad():
            b1p, b2p = float(self.powers[0]), float(self.powers[1])
            R.tf_adam_update(self.params.flat, grads, self.m.flat, self.v.flat, b1p, b2p,
                             self.lr, self.beta1, self.beta2, self.eps)
            self.powers[0] = self.powers[0] * self.beta1
            self.powers[1] = self.powers[1] * self.beta2

    # ------------------------------------------------------------------ ckpt
    def tf_slot_tensors(self) -> "OrderedDict[str, torch.Tensor]":
        out = OrderedDict()
        for name in self.params.names():
            out[name + "/Adam"] = self.m[name]
            out[name + "/Adam_1"] = self.v[name]
        out["beta1_power" + self.power_suffix] = self.powers[0:1]
        out["beta2_power" + self.power_suffix] = self.powers[1:2]
        return out

    def load_tf_slots(self, sd: Dict[str, torch.Tensor]) -> bool:
        """Restore slots; returns False (and zero-initialises, t=0) when the checkpoint
        has no optimiser state, as reference-written checkpoints do."""
        key1 = "beta1_power" + self.power_suffix
        if key1 not in sd:
            with torch.no_grad():
                self.m.flat.zero_()
                self.v.flat.zero_()
                self.powers.copy_(torch.tensor([self.beta1, self.beta2], dtype=torch.float32))
            return False
        with torch.no_grad():
            for name in self.params.names():
                self.m[name].copy_(torch.as_tensor(sd[name + "/Adam"]).to(self.m[name]))
                self.v[name].copy_(torch.as_tensor(sd[name + "/Adam_1"]).to(self.v[name]))
            self.powers[0] = float(torch.as_tensor(sd[key1]).reshape(-1)[0])
            self.powers[1] = float(torch.as_tensor(sd["beta2_power" + self.power_suffix]).reshape(-1)[0])
        return True
