"""Engine selection: the fused HIP engine on an MI355X (bf16, fp16 or fp32), the reference
(PyTorch autograd) engine on the CPU or when asked for explicitly.

Both expose the same small interface used by the trainer and ``bench.py``:
``set_synthetic_batch(real)``, ``set_batch(real)``, ``train_step()``, ``last_losses()``,
``model`` (parameters + BN state), ``opt_d``/``opt_g`` (TF-Adam state), ``global_step``.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..models.config import DCGANConfig
from ..models.dcgan import DCGAN
from ..parallel import dist as D
from .reference_step import ReferenceStep


class ReferenceEngine:
    """Autograd reference step (PyTorch ops) + gloo/RCCL gradient averaging."""

    name = "reference"
    dtype_name = "fp32"

    def __init__(self, cfg: DCGANConfig, batch_size: int, device: torch.device, seed: int = 0,
                 lr: float = 2e-4, beta1: float = 0.5, zero_debias: bool = False, rank: int = 0,
                 world: int = 1, z_seed: Optional[int] = None, **_):
        self.cfg = cfg
        self.batch_size = batch_size
        self.device = device
        self.model = DCGAN(cfg, device=device, seed=seed, zero_debias=zero_debias)
        self.world = world
        if world > 1:
            D.broadcast_tensors([self.model.g.flat, self.model.d.flat, self.model.g_bn.flat,
                                 self.model.d_bn.flat])
        self.step_impl = ReferenceStep(self.model, lr, beta1, grad_hook=self._allreduce if world > 1 else None)
        self.opt_d, self.opt_g = self.step_impl.opt_d, self.step_impl.opt_g
        self.z_gen = torch.Generator(device=device if device.type == "cuda" else "cpu")
        self.z_gen.manual_seed((z_seed if z_seed is not None else seed) + 7919 * rank + 1)
        self._real = None
        self._losses: Dict[str, float] = {}

    def _allreduce(self, which: str, flat: torch.Tensor) -> None:
        D.all_reduce_mean_(flat)

    @property
    def global_step(self) -> int:
        return self.step_impl.global_step

    @global_step.setter
    def global_step(self, v: int) -> None:
        self.step_impl.global_step = int(v)

    def set_synthetic_batch(self, real: torch.Tensor) -> None:
        self._real = real.to(self.device, torch.float32)

    def set_batch(self, real: torch.Tensor) -> None:
        self._real = real.to(self.device, torch.float32, non_blocking=True)

    def sample_z(self, n: int) -> torch.Tensor:
        return torch.rand(n, self.cfg.z_dim, generator=self.z_gen, device=self.device) * 2 - 1

    def train_step(self) -> None:
        z = self.sample_z(self._real.shape[0])
        self._last_z = z
        self._losses = self.step_impl.step(self._real, z)

    def activations(self) -> "Dict[str, torch.Tensor]":
        """Re-run the last step's forward (pre-update weights are gone; uses current ones,
        no EMA update) and return the summary tensors."""
        from collections import OrderedDict
        rec: Dict[str, torch.Tensor] = {}
        B = self._real.shape[0]
        with torch.no_grad():
            out = self.step_impl.forward_losses(self._real, self._last_z, update_ema=False, record=rec)
        a = OrderedDict()
        a["z"] = self._last_z
        a["d"] = torch.sigmoid(out["logits_real"])
        a["d_"] = torch.sigmoid(out["logits_fake"])
        a["G"] = out["fake"]
        a["g_h0_relu"] = rec["g_h0"]
        gl = self.cfg.g_layers()
        for L in gl[:-1]:
            a[L.name + "_relu"] = rec[L.name]
        a[gl[-1].name] = rec[gl[-1].name]
        for L in self.cfg.d_layers():
            a[L.name] = rec[L.name][:B]
        a[self.cfg.d_lin_name] = out["logits_real"]
        return a

    def last_losses(self) -> Dict[str, float]:
        return dict(self._losses)

    def sampler(self, z: torch.Tensor) -> torch.Tensor:
        return self.model.sampler(z.to(self.device))

    def eval_losses(self, real: torch.Tensor, z: torch.Tensor) -> Dict[str, float]:
        """Sample-time d_loss/g_loss (image_train.py:181-184) without mutating BN EMAs."""
        with torch.no_grad():
            out = self.step_impl.forward_losses(real.to(self.device, torch.float32), z.to(self.device),
                                                update_ema=False)
        return {"d_loss": float(out["d_loss"]), "g_loss": float(out["g_loss"])}

    def sync_state_for_checkpoint(self) -> None:
        pass

    def sync_bn_state(self) -> None:
        """Average the BN moving averages over ranks (collective; every rank must call it).
        Each rank tracks its own local-batch statistics; the reference's shared PS copy saw
        every worker's updates, which the mean over ranks approximates."""
        D.all_reduce_mean_(self.model.g_bn.flat)
        D.all_reduce_mean_(self.model.d_bn.flat)


def build_engine(cfg: DCGANConfig, batch_size: int, device: torch.device, engine: str = "auto",
                 dtype: str = "bf16", seed: int = 0, rank: int = 0, world: int = 1, graph: bool = True,
                 allreduce_dtype: str = "fp32", lr: float = 2e-4, beta1: float = 0.5,
                 zero_debias: bool = False, bucket_mb: float = 32.0):
    if engine == "auto":  # every dtype (bf16 / fp16 / fp32) runs on the HIP kernels on an MI355X
        engine = "hip" if device.type == "cuda" else "reference"
    if engine == "reference":
        return ReferenceEngine(cfg, batch_size, device, seed=seed, lr=lr, beta1=beta1,
                               zero_debias=zero_debias, rank=rank, world=world)
    if engine == "hip":
        from .hip_engine import HipEngine
        return HipEngine(cfg, batch_size, device, dtype=dtype, seed=seed, lr=lr, beta1=beta1,
                         zero_debias=zero_debias, rank=rank, world=world, graph=graph,
                         allreduce_dtype=allreduce_dtype, bucket_mb=bucket_mb)
    raise ValueError("unknown engine %r" % engine)
