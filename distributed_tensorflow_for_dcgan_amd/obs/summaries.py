"""The reference's TensorBoard summaries, computed from engine state on summary steps only.

On the HIP engine the histograms and zero fractions are reduced on the device
(``HipEngine.device_summaries``, csrc/hip/summary.hip): only per-tensor statistics rows cross
to the host, not the activations and weights themselves; the other engines bin on the host.

Reference sources: scalars ``d_loss_real, d_loss_fake, g_loss, d_loss`` (``image_train.py:98-101``);
histograms ``z, d, d_`` and image ``G`` (max 3) (``:86-89``); a histogram per trainable variable
(``:114-115``); per-layer ``<name>/activations`` histograms and ``<name>/sparsity`` (zero
fraction) scalars (``distriubted_model.py:75-80``); and what the TF runtime adds on its own:
``global_step/sec`` (Supervisor) and input-queue fullness.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from .events import SummaryWriter


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().float().cpu().numpy()


def collect(engine, losses: Dict[str, float], steps_per_sec: Optional[float] = None,
            loader_stats: Optional[dict] = None, max_images: int = 3) -> List[bytes]:
    S = SummaryWriter
    vals: List[bytes] = []
    for k in ("d_loss_real", "d_loss_fake", "g_loss", "d_loss"):
        if k in losses:
            vals.append(S.scalar(k, losses[k]))
    acts = engine.activations()
    if hasattr(engine, "device_summaries"):  # histograms / sparsity reduced on the device (summary.hip)
        rows = engine.device_summaries()
        if "G" in acts:
            g = (_np(acts["G"][:max_images]) + 1.0) / 2.0
            for i in range(g.shape[0]):
                vals.append(S.image("G/image/%d" % i if g.shape[0] > 1 else "G/image", g[i]))
        for name, row in rows.items():
            vals.append(S.histogram_from_stats(name, row))
            if name.endswith("/activations"):
                vals.append(S.scalar(name[:-len("/activations")] + "/sparsity", float(row[5] / max(1.0, row[2]))))
        _tail(vals, steps_per_sec, loader_stats)
        return vals
    if "z" in acts:
        vals.append(S.histogram("z", _np(acts["z"])))
    if "d" in acts:
        vals.append(S.histogram("d", _np(acts["d"])))
    if "d_" in acts:
        vals.append(S.histogram("d_", _np(acts["d_"])))
    if "G" in acts:
        g = (_np(acts["G"][:max_images]) + 1.0) / 2.0
        for i in range(g.shape[0]):
            vals.append(S.image("G/image/%d" % i if g.shape[0] > 1 else "G/image", g[i]))
    for name, t in acts.items():
        if name in ("z", "d", "d_", "G"):
            continue
        a = _np(t)
        vals.append(S.histogram(name + "/activations", a))
        vals.append(S.scalar(name + "/sparsity", float((a == 0).mean())))
    for name, t in engine.model.all_named_variables().items():
        vals.append(S.histogram(name, _np(t)))
    _tail(vals, steps_per_sec, loader_stats)
    return vals


def _tail(vals: List[bytes], steps_per_sec: Optional[float], loader_stats: Optional[dict]) -> None:
    S = SummaryWriter
    if steps_per_sec is not None:
        vals.append(S.scalar("global_step/sec", steps_per_sec))
    if loader_stats and "fraction_of_capacity_full" in loader_stats:
        vals.append(S.scalar("shuffle_batch/fraction_over_min_after_dequeue",
                             float(loader_stats["fraction_of_capacity_full"])))
