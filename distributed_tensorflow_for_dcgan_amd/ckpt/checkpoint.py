"""Checkpoint save / restore with the reference's directory layout and variable names.

Reference behaviour: ``tf.train.Supervisor(logdir=checkpoint_dir,
save_model_secs=600)`` on the chief writes ``checkpoint_dir/model.ckpt-<global_step>`` plus the
``checkpoint`` text index, keeps the last 5, and restores the latest on start
(``image_train.py:123-146,233-245``). Its Saver is built before the optimisers, so Adam state
is NOT saved and a restart fails the readiness check.

Here (a compatible superset):

* same prefix naming, same ``checkpoint`` text-proto index (written last, atomically);
* TF V2 tensor-bundle files (``.index`` + ``.data-00000-of-00001``, see ``tf_bundle``);
* variables under their TF names and TF layouts (HWIO conv, [kh,kw,out,in] deconv,
  [in,out] linear with NHWC flatten order), ``Variable`` = global_step (int32), BN moving
  averages under ``<scope>/moments/Squeeze[_1]/ExponentialMovingAverage``;
* PLUS the optimiser state under TF's slot names (``<var>/Adam``, ``<var>/Adam_1``,
  ``beta1_power``/``beta2_power`` for D, ``..._1`` for G) so resume is exact; restore
  tolerates reference-style checkpoints without it (Adam restarts at t = 0);
* a ``.json`` sidecar with the model config / data position (not read by TF).
"""
from __future__ import annotations

import json
import os
import re
import time
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import torch

from . import tf_bundle

INDEX_FILE = "checkpoint"


def _q(s: str) -> str:
    return '"%s"' % s.replace("\\", "\\\\").replace('"', '\\"')


def write_index(ckpt_dir: str, latest: str, all_paths: List[str]) -> None:
    lines = ["model_checkpoint_path: %s" % _q(latest)]
    lines += ["all_model_checkpoint_paths: %s" % _q(p) for p in all_paths]
    tmp = os.path.join(ckpt_dir, INDEX_FILE + ".tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(ckpt_dir, INDEX_FILE))


def read_index(ckpt_dir: str) -> Optional[Dict[str, object]]:
    """Parse the ``checkpoint`` text proto (``tf.train.get_checkpoint_state``)."""
    path = os.path.join(ckpt_dir, INDEX_FILE)
    if not os.path.exists(path):
        return None
    latest, allp = None, []
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths)\s*:\s*"(.*)"\s*$', line)
            if not m:
                continue
            val = m.group(2).encode().decode("unicode_escape")
            if m.group(1) == "model_checkpoint_path":
                latest = val
            else:
                allp.append(val)
    if latest is None:
        return None
    return {"model_checkpoint_path": latest, "all_model_checkpoint_paths": allp}


def latest_checkpoint(ckpt_dir: str) -> Optional[str]:
    st = read_index(ckpt_dir)
    if not st:
        return None
    p = st["model_checkpoint_path"]
    if not os.path.isabs(p):
        p = os.path.join(ckpt_dir, p)
    if os.path.exists(p + ".index"):
        return p
    return None


BN_STEPS_KEYS = ("g_bn/ExponentialMovingAverage/local_step", "d_bn/ExponentialMovingAverage/local_step")


def collect_state(engine) -> "OrderedDict[str, np.ndarray]":
    """TF-named numpy tensors of everything a resume needs."""
    engine.sync_state_for_checkpoint()
    m = engine.model
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for k, v in m.g.tensors.items():
        out[k] = v.detach().cpu().numpy().astype(np.float32)
    for k, v in m.d.tensors.items():
        out[k] = v.detach().cpu().numpy().astype(np.float32)
    out["Variable"] = np.array(int(engine.global_step), dtype=np.int32)
    for k, v in m.g_bn.tf_names().items():
        out[k] = v.detach().cpu().numpy().astype(np.float32)
    for k, v in m.d_bn.tf_names().items():
        out[k] = v.detach().cpu().numpy().astype(np.float32)
    # moving-average update counts (the --bn_zero_debias divisor 1 - decay^t; TF keeps a
    # local_step per average for the same purpose)
    out[BN_STEPS_KEYS[0]] = m.g_bn.steps.numpy().astype(np.float64)
    out[BN_STEPS_KEYS[1]] = m.d_bn.steps.numpy().astype(np.float64)
    for opt in (engine.opt_d, engine.opt_g):
        for k, v in opt.tf_slot_tensors().items():
            a = v.detach().cpu().numpy().astype(np.float32)
            out[k] = a.reshape(()) if k.startswith("beta") else a
    return out


def apply_state(engine, sd: Dict[str, np.ndarray], strict: bool = True) -> Dict[str, object]:
    m = engine.model
    info: Dict[str, object] = {}
    tsd = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}
    missing = m.g.load_state_dict(tsd, strict=False) + m.d.load_state_dict(tsd, strict=False)
    if strict and missing:
        raise KeyError("checkpoint lacks variables: %s" % missing)
    with torch.no_grad():
        for names in (m.g_bn.tf_names(), m.d_bn.tf_names()):
            for k, v in names.items():
                if k in tsd:
                    v.copy_(tsd[k].to(v.dtype).reshape(v.shape))
        # EMA update counts: saved ones, else one update per synchronous step (older checkpoints)
        step_now = int(np.asarray(sd["Variable"]).reshape(-1)[0]) if "Variable" in sd else 0
        for key, bn in zip(BN_STEPS_KEYS, (m.g_bn, m.d_bn)):
            if key in tsd and tsd[key].numel() == bn.steps.numel():
                bn.steps.copy_(tsd[key].to(torch.float64).reshape(bn.steps.shape))
            else:
                bn.steps.fill_(float(step_now))
    info["adam_d"] = engine.opt_d.load_tf_slots(tsd)
    info["adam_g"] = engine.opt_g.load_tf_slots(tsd)
    if "Variable" in tsd:
        engine.global_step = int(np.asarray(sd["Variable"]).reshape(-1)[0])
    info["global_step"] = int(engine.global_step)
    if hasattr(engine, "after_state_load"):
        engine.after_state_load()
    return info


class CheckpointManager:
    """Chief-side timed checkpointing (``--save_model_secs``) with keep-last-N."""

    def __init__(self, ckpt_dir: str, keep: int = 5, save_secs: float = 600.0, prefix: str = "model.ckpt"):
        self.dir = ckpt_dir
        self.keep = max(1, int(keep))
        self.save_secs = float(save_secs)
        self.prefix = prefix
        self.last_save = time.time()
        os.makedirs(ckpt_dir, exist_ok=True)

    def save(self, engine, extra: Optional[Dict[str, object]] = None) -> str:
        step = int(engine.global_step)
        name = "%s-%d" % (self.prefix, step)
        path = os.path.join(self.dir, name)
        tf_bundle.write_bundle(path, collect_state(engine))
        meta = {"global_step": step, "time": time.time()}
        cfg = getattr(engine, "cfg", None)
        if cfg is not None:
            meta["config"] = {k: getattr(cfg, k) for k in cfg.__dataclass_fields__}
        if extra:
            meta.update(extra)
        with open(path + ".json.tmp", "w") as f:
            json.dump(meta, f, indent=1, default=str)
        os.replace(path + ".json.tmp", path + ".json")
        st = read_index(self.dir)
        allp = [p for p in (st["all_model_checkpoint_paths"] if st else []) if p != name] + [name]
        for old in allp[:-self.keep]:
            for suf in (".index", ".data-00000-of-00001", ".json", ".meta"):
                try:
                    os.remove(os.path.join(self.dir, old + suf))
                except FileNotFoundError:
                    pass
        allp = allp[-self.keep:]
        write_index(self.dir, name, allp)  # index last: a crash never points at a partial file
        self.last_save = time.time()
        return path

    def maybe_save(self, engine, now: Optional[float] = None) -> Optional[str]:
        now = time.time() if now is None else now
        if self.save_secs > 0 and now - self.last_save >= self.save_secs:
            return self.save(engine)
        return None

    def restore_latest(self, engine) -> Optional[Dict[str, object]]:
        p = latest_checkpoint(self.dir)
        if p is None:
            return None
        sd = tf_bundle.read_bundle(p)
        info = apply_state(engine, sd, strict=True)
        info["path"] = p
        return info
