"""``image_train.py``-compatible flag system.

Reproduces the 22 ``tf.app.flags`` definitions of the reference
(``/root/reference/image_train.py:10-40``) with the same names, types, defaults and
syntax (``--name=value``, ``--name value``, bare ``--bool``, ``--nobool``), and wires
every one of them for real (the reference ignores most of them).
New, additive flags (dtype, synthetic data, max_steps, seed, gf/df dims, DDP knobs,
profiling) are registered in the same table so ``FLAGS.__flags``-style pprint shows
the full effective configuration (reference ``image_train.py:223``).
"""
from __future__ import annotations

import argparse
import math
import os
import sys
from typing import Any, Dict, List, Optional, Sequence, Tuple

# (name, type, default, help)  -- reference flags first, in reference order.
REFERENCE_FLAGS: List[Tuple[str, str, Any, str]] = [
    ("epoch", "int", 25, "Epoch to train [25]"),
    ("learning_rate", "float", 0.0002, "Learning rate of for adam [0.0002]"),
    ("beta1", "float", 0.5, "Momentum term of adam [0.5]"),
    ("train_size", "int", math.inf, "The size of train images [np.inf]"),
    ("batch_size", "int", 64, "The size of batch images [64]"),
    ("image_size", "int", 108, "The size of image to use (will be center cropped) [108]"),
    ("output_size", "int", 64, "The size of the output images to produce [64]"),
    ("c_dim", "int", 3, "Dimension of image color. [3]"),
    ("dataset", "str", "celebA", "The name of dataset [celebA, mnist, lsun]"),
    ("checkpoint_dir", "str", "checkpoint", "Directory name to save the checkpoints [checkpoint]"),
    ("sample_dir", "str", "samples", "Directory name to save the image samples [samples]"),
    ("is_train", "bool", False, "True for training, False for testing [False]"),
    ("is_crop", "bool", False, "True for training, False for testing [False]"),
    ("visualize", "bool", False, "True for visualizing, False for nothing [False]"),
    ("data_dir", "str", "train", "dir for train set"),
    ("sample_image_dir", "str", "sample_data", "dir for train set"),
    ("ps_hosts", "str", "", "Comma-separated list of hostname:port pairs"),
    ("worker_hosts", "str", "", "Comma-separated list of hostname:port pairs"),
    ("job_name", "str", "", "One of 'ps', 'worker'"),
    ("task_index", "int", 0, "Index of task within the job"),
    ("log_device_placement", "bool", True, "whether to log the device placement"),
    ("save_summaries_secs", "int", 10, "Save summaries interval seconds."),
]

# Additive flags of this framework (not in the reference).
EXTRA_FLAGS: List[Tuple[str, str, Any, str]] = [
    ("dtype", "str", "bf16", "compute dtype: bf16 | fp16 (dynamic loss scaling) | fp32 (reference precision)"),
    ("device", "str", "auto", "auto | cpu | cuda (cuda == the local MI355X via HIP)"),
    ("synthetic", "bool", False, "use synthetic images of the configured shape instead of TFRecords"),
    ("max_steps", "int", 1200000, "stop after this many global steps (reference hard-codes 1,200,000)"),
    ("seed", "int", 0, "base RNG seed; rank r uses seed + r for z and data order"),
    ("gf_dim", "int", 64, "generator base channel count"),
    ("df_dim", "int", 64, "discriminator base channel count"),
    ("z_dim", "int", 100, "latent dimension"),
    ("depth", "int", 0, "number of stride-2 stages (0 = auto from output_size)"),
    ("max_channels", "int", 0, "cap on per-layer channels (0 = no cap)"),
    ("save_model_secs", "float", 600.0,"chief checkpoint interval in seconds (reference Supervisor default 600)"),
    ("keep_checkpoints", "int", 5, "number of checkpoints to keep (TF Saver default 5)"),
    ("sample_every", "int", 100, "sample when global_step %% sample_every == 1 (reference: 100)"),
    ("engine", "str", "auto", "auto | hip | reference : which training step implementation"),
    ("graph", "bool", False, "replay the HIP training step as hipGraph(s) instead of the C++ launch replay "
                              "(measured 1-3 %% slower: profiles/r5/ab_eager_vs_graph_r5.txt)"),
    ("bucket_mb", "float", 32.0, "gradient all-reduce bucket size in MiB (HIP engine: one call per overlap window)"),
    ("allreduce_dtype", "str", "fp32", "gradient all-reduce wire dtype: fp32 | bf16"),
    ("shard_data", "bool", True, "give every rank a disjoint shard of the input files"),
    ("shuffle_buffer", "int", 10776, "shuffle-buffer min_after_dequeue (reference: 10% of 107,766)"),
    ("loader_threads", "int", 16, "native TFRecord reader threads (reference: 16 queue runners)"),
    ("bn_zero_debias", "bool", False, "apply TF>=0.12 zero-debiasing to BN moving averages"),
    ("profile_steps", "str", "", "a:b -> run torch.profiler over global steps [a, b)"),
    ("log_every", "int", 1, "print the step line every N steps (reference: every step)"),
    ("summaries", "bool", True, "write TensorBoard event files on the chief"),
    ("verbose", "bool", False, "verbose device / placement logging"),
    ("timing", "bool", False, "per-phase GPU timers (fwd+D bwd / G bwd / optimiser / comm) on log steps"),
    ("check_sync_every", "int", 0, "every N steps assert that parameters are bit-identical across ranks"),
    ("cache_on_device", "bool", False, "decode the whole TFRecord dataset once into GPU memory (288 GB HBM)"),
    ("collective_timeout", "float", 600.0, "seconds before a hung collective is an error (RCCL watchdog)"),
    ("num_samples", "int", 64, "images per grid in sample-only mode (--nois_train)"),
]

ALL_FLAGS = REFERENCE_FLAGS + EXTRA_FLAGS


class Flags:
    """Attribute bag that also exposes ``__flags`` like TF 0.x's ``FLAGS``."""

    def __init__(self, values: Dict[str, Any], explicit: Optional[Sequence[str]] = None):
        object.__setattr__(self, "_values", dict(values))
        object.__setattr__(self, "_explicit", frozenset(explicit or ()))

    def explicitly_set(self, name: str) -> bool:
        """True when the flag appeared on the command line (``--x``, ``--x=v``, ``--nox``)."""
        return name in object.__getattribute__(self, "_explicit")

    def __getattr__(self, name: str) -> Any:
        values = object.__getattribute__(self, "_values")
        if name == "__flags":
            return dict(values)
        if name in values:
            return values[name]
        raise AttributeError(name)

    def __setattr__(self, name: str, value: Any) -> None:
        self._values[name] = value

    def as_dict(self) -> Dict[str, Any]:
        return dict(self._values)

    def __repr__(self) -> str:  # pragma: no cover - cosmetic
        return "Flags(%r)" % (self._values,)


def _parse_bool(text: str) -> bool:
    low = text.strip().lower()
    if low in ("1", "true", "t", "yes", "y"):
        return True
    if low in ("0", "false", "f", "no", "n"):
        return False
    raise argparse.ArgumentTypeError("invalid boolean value: %r" % text)


def _parse_int(text: str) -> Any:
    low = text.strip().lower()
    if low in ("inf", "np.inf", "infinity"):
        return math.inf
    return int(text)


_CONVERTERS = {"int": _parse_int, "float": float, "str": str, "bool": _parse_bool}


def build_parser(defaults_override: Optional[Dict[str, Any]] = None) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        prog="image_train.py",
        description="MI355X-native distributed DCGAN training (image_train.py-compatible flags)",
        allow_abbrev=False,
    )
    overrides = defaults_override or {}
    for name, typ, default, help_text in ALL_FLAGS:
        default = overrides.get(name, default)
        if typ == "bool":
            # --name, --name=true/false, --noname  (absl/tf.app.flags semantics)
            p.add_argument("--" + name, dest=name, nargs="?", const=True, default=default,
                           type=_parse_bool, help=help_text)
            p.add_argument("--no" + name, dest=name, action="store_false", help=argparse.SUPPRESS)
        else:
            p.add_argument("--" + name, dest=name, type=_CONVERTERS[typ], default=default, help=help_text)
    return p


def parse_flags(argv: Optional[Sequence[str]] = None,
                defaults_override: Optional[Dict[str, Any]] = None) -> Flags:
    """Parse ``argv`` (without the program name). Unknown flags are an error."""
    parser = build_parser(defaults_override)
    argv = list(argv) if argv is not None else sys.argv[1:]
    ns = parser.parse_args(argv)
    names = {n for n, _, _, _ in ALL_FLAGS}
    explicit = set()
    for tok in argv:
        if tok.startswith("--"):
            key = tok[2:].split("=", 1)[0]
            if key in names:
                explicit.add(key)
            elif key.startswith("no") and key[2:] in names:
                explicit.add(key[2:])
    return Flags(vars(ns), explicit)


# --dataset presets (carpedm20/DCGAN-tensorflow naming, which the reference's flag help lists:
# "celebA, mnist, lsun"): image shape for the flags the command line did not set, and the
# ``data/<dataset>`` directory when --data_dir is left at its default and that directory exists.
DATASET_PRESETS: Dict[str, Dict[str, Any]] = {
    "celebA": {"output_size": 64, "c_dim": 3},
    "lsun": {"output_size": 64, "c_dim": 3},
    "mnist": {"output_size": 28, "c_dim": 1},
    "cifar10": {"output_size": 32, "c_dim": 3},
}


def apply_dataset_preset(flags: Flags) -> Dict[str, Any]:
    """Apply the --dataset preset in place; returns what it changed (name -> value). Unknown
    names are kept (they label checkpoints / logs) and change nothing."""
    changed: Dict[str, Any] = {}
    name = str(flags.dataset)
    preset = DATASET_PRESETS.get(name) or {k.lower(): v for k, v in DATASET_PRESETS.items()}.get(name.lower())
    for k, v in (preset or {}).items():
        if not flags.explicitly_set(k) and getattr(flags, k) != v:
            setattr(flags, k, v)
            changed[k] = v
    if not flags.explicitly_set("data_dir"):
        d = os.path.join("data", name)
        if not os.path.isdir(flags.data_dir) and os.path.isdir(d):
            flags.data_dir = d
            changed["data_dir"] = d
    return changed


def default_flags(**overrides: Any) -> Flags:
    values = {name: default for name, _, default, _ in ALL_FLAGS}
    for k, v in overrides.items():
        if k not in values:
            raise KeyError("unknown flag %r" % k)
        values[k] = v
    return Flags(values)


def cluster_from_flags(flags: Flags) -> Dict[str, Any]:
    """Map the reference's cluster flags onto a torch.distributed rendezvous.

    torchrun-style env vars (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT) win. Without them,
    ``--worker_hosts=h0:p0,h1:p1,...`` + ``--task_index=i`` give world_size = #workers,
    rank = i and master = the first worker (the chief, reference ``image_train.py:123``).
    ``--job_name=ps`` has no meaning in synchronous DDP (there is no parameter server);
    the caller reports that and exits 0.
    """
    env = os.environ
    if "RANK" in env and "WORLD_SIZE" in env:
        return {
            "rank": int(env["RANK"]),
            "world_size": int(env["WORLD_SIZE"]),
            "local_rank": int(env.get("LOCAL_RANK", env["RANK"])),
            "master_addr": env.get("MASTER_ADDR", "127.0.0.1"),
            "master_port": int(env.get("MASTER_PORT", "29500")),
            "source": "env",
        }
    workers = [w.strip() for w in flags.worker_hosts.split(",") if w.strip()] if flags.worker_hosts else []
    if len(workers) > 1:
        host, _, port = workers[0].rpartition(":")
        if flags.task_index < 0 or flags.task_index >= len(workers):
            raise ValueError("--task_index=%d out of range for %d workers" % (flags.task_index, len(workers)))
        # one process per GPU: this worker's GPU is its index among the workers listed for the
        # same host (reference launches N workers on one box as N --worker_hosts entries)
        my_host = workers[flags.task_index].rpartition(":")[0]
        local = sum(1 for w in workers[:flags.task_index] if w.rpartition(":")[0] == my_host)
        return {
            "rank": flags.task_index,
            "world_size": len(workers),
            "local_rank": int(env.get("LOCAL_RANK", str(local))),
            "master_addr": host or "127.0.0.1",
            "master_port": int(port or 29500),
            "source": "worker_hosts",
        }
    return {"rank": 0, "world_size": 1, "local_rank": 0, "master_addr": "127.0.0.1",
            "master_port": 29500, "source": "single"}
