"""``image_train.py``-compatible training driver (reference ``image_train.py:51-249``).

Loop per step: next batch (native loader, already on the device) -> engine step (G fwd,
D(real)+D(fake), 3 losses, backward, gradient all-reduce over RCCL when W > 1, two TF-Adam
updates) -> the reference's log line -> chief-only TensorBoard summaries every
``--save_summaries_secs`` -> chief-only sample grid when ``global_step % 100 == 1`` -> chief-only
checkpoint every ``--save_model_secs``; auto-resume from the newest checkpoint on start.

Deliberate differences: synchronous data parallelism instead of the
asynchronous parameter server (``--job_name=ps`` exits with a notice), every flag is honoured,
epochs count W*B images per global step, the sample-time losses do not mutate the BN moving
averages, samples go to ``--sample_dir``, optimiser state is checkpointed.
"""
from __future__ import annotations

import math
import os
import pprint
import sys
import time
from typing import List, Optional

import numpy as np
import torch

from ..ckpt.checkpoint import CheckpointManager
from ..data.pipeline import make_source
from ..engine.factory import build_engine
from ..models.config import config_from_flags
from ..obs import images as IM
from ..obs import summaries as SUM
from ..obs.events import SummaryWriter
from ..parallel import dist as D
from ..utils.flags import Flags, apply_dataset_preset, cluster_from_flags

STEP_LINE = "Epoch: [%2d] step: [%2d] time: %4.4f, d_loss: %.8f, g_loss: %.8f"
SYNC_EVERY = 10  # steps between collective checks of the chief's time-based save decision
LOSS_KEYS = ("d_loss_real", "d_loss_fake", "g_loss", "d_loss")


class AsyncLossLog:
    """The reference prints its step line after every ``sess.run`` (image_train.py:160-162),
    which on a GPU engine means a host sync per step. Here the device loss vector is copied into
    a small ring of pinned host buffers without blocking (``non_blocking`` copy + event); a line
    is printed once its copy has landed -- normally one step later -- so the training stream
    never waits for the host. Engines without a device loss tensor are read synchronously."""

    def __init__(self, engine, device, depth: int = 8):
        self.engine = engine
        self.async_ = device.type == "cuda" and hasattr(engine, "losses_tensor")
        self.pending = []   # (meta, event, pinned buffer), oldest first
        self.landed = []    # (meta, values) taken out of a full ring
        self.free = ([torch.empty(4, dtype=torch.float32, pin_memory=True) for _ in range(depth)]
                     if self.async_ else [])

    def push(self, meta) -> None:
        if not self.async_:
            L = self.engine.last_losses()
            self.landed.append((meta, [L[k] for k in LOSS_KEYS]))
            return
        if not self.free:  # ring full (the GPU is far behind): retire the oldest copy
            m, ev, buf = self.pending.pop(0)
            ev.synchronize()
            self.landed.append((m, buf.tolist()))
            self.free.append(buf)
        buf = self.free.pop()
        buf.copy_(self.engine.losses_tensor(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((meta, ev, buf))

    def ready(self, flush: bool = False):
        """(meta, losses dict) of every landed entry, oldest first (all of them when flush)."""
        out = [(m, dict(zip(LOSS_KEYS, v))) for m, v in self.landed]
        self.landed = []
        while self.pending:
            meta, ev, buf = self.pending[0]
            if flush:
                ev.synchronize()
            elif not ev.query():
                break
            self.pending.pop(0)
            out.append((meta, dict(zip(LOSS_KEYS, buf.tolist()))))
            self.free.append(buf)
        return out


def _device(flags: Flags, local_rank: int) -> torch.device:
    want = flags.device
    if want == "cpu" or (want == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    return torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))


def placement_report(engine, device, rank: int, world: int) -> List[str]:
    """--log_device_placement (reference ``image_train.py:36``, defined there but never passed to
    a session): where this rank's work runs -- the TF-style device name, the HIP device, the
    process group, and the engine's streams / graphs."""
    lines = []
    if device.type == "cuda":
        pr = torch.cuda.get_device_properties(device)
        lines.append("/job:worker/replica:0/task:%d/device:GPU:%d -> HIP device %d: %s, %d CUs, %.0f GiB, arch %s"
                     % (rank, device.index or 0, device.index or 0, pr.name, pr.multi_processor_count,
                        pr.total_memory / 2 ** 30, getattr(pr, "gcnArchName", "?")))
    else:
        lines.append("/job:worker/replica:0/task:%d/device:CPU:0 -> host CPU" % rank)
    if D.is_initialized():
        import torch.distributed as tdist
        lines.append("process group: backend %s, rank %d of %d" % (tdist.get_backend(), rank, tdist.get_world_size()))
    else:
        lines.append("process group: none (single process, world %d)" % world)
    rep = getattr(engine, "placement", None)
    if callable(rep):
        lines.extend(rep())
    return ["[placement] " + l for l in lines]


def run(flags: Flags, out=None) -> int:
    out = sys.stdout if out is None else out
    preset = apply_dataset_preset(flags)
    pprint.pprint(flags.as_dict(), stream=out)
    if preset:
        print("--dataset=%s preset: %s" % (flags.dataset, ", ".join("%s=%s" % kv for kv in sorted(preset.items()))),
              file=out)
        if "output_size" in preset or "c_dim" in preset:
            # the reference ignores --dataset and always builds 64x64x3 (distriubted_model.py:7-11)
            print("WARNING: --dataset=%s changed the model shape to %dx%dx%d; the reference always trains "
                  "64x64x3. Records of another shape fail to decode (image_raw size check); pass "
                  "--output_size/--c_dim to override." % (flags.dataset, flags.output_size, flags.output_size,
                                                         flags.c_dim), file=out)
    if flags.job_name == "ps":
        print("--job_name=ps: this framework trains with synchronous data parallelism over RCCL; "
              "there is no parameter server to run. Launch one worker per GPU instead "
              "(e.g. torchrun --nproc-per-node N image_train.py ...).", file=out)
        return 0
    if flags.job_name not in ("", "worker"):
        raise SystemExit("unknown --job_name=%r (expected 'worker' or 'ps')" % flags.job_name)
    os.makedirs(flags.checkpoint_dir, exist_ok=True)
    os.makedirs(flags.sample_dir, exist_ok=True)

    cl = cluster_from_flags(flags)
    rank, world = cl["rank"], cl["world_size"]
    device = _device(flags, cl["local_rank"])
    if device.type == "cuda":
        torch.cuda.set_device(device)
    D.init_distributed(world, rank, device, cl["master_addr"], cl["master_port"],
                       timeout_s=float(flags.collective_timeout))
    chief = rank == 0
    cfg = config_from_flags(flags)
    B = int(flags.batch_size)
    shape = (cfg.output_size, cfg.output_size, cfg.c_dim)
    if flags.verbose:
        print("device %s rank %d/%d local_rank %d (%s) engine %s" % (device, rank, world, cl["local_rank"],
                                                                   cl["source"], flags.engine), file=out, flush=True)

    engine = build_engine(cfg, B, device, engine=flags.engine, dtype=flags.dtype, seed=int(flags.seed), rank=rank,
                          world=world, graph=bool(flags.graph), allreduce_dtype=flags.allreduce_dtype,
                          lr=float(flags.learning_rate), beta1=float(flags.beta1),
                          zero_debias=bool(flags.bn_zero_debias), bucket_mb=float(flags.bucket_mb))
    if flags.log_device_placement:
        for line in placement_report(engine, device, rank, world):
            print(line, file=out, flush=True)
    ckpt = CheckpointManager(flags.checkpoint_dir, keep=int(flags.keep_checkpoints),
                             save_secs=float(flags.save_model_secs))
    info = ckpt.restore_latest(engine)
    if chief:
        print(" [*] Reading checkpoints...", file=out)
        print("load success! (%s, global_step %d)" % (info["path"], info["global_step"]) if info
              else "load failed!!", file=out)
        if info and not (info.get("adam_d") and info.get("adam_g")):
            print("note: checkpoint has no optimiser state (reference-style); Adam restarts at t=0", file=out)

    if flags.explicitly_set("is_train") and not flags.is_train:
        try:
            return _test_mode(engine, flags, cfg, B, device, info, chief, out)
        finally:
            D.barrier()
            D.shutdown()
    if bool(flags.timing) and hasattr(engine, "enable_timing"):
        engine.enable_timing()

    edt = getattr(engine, "dtype_name", None)
    source = make_source(flags, B, shape, device, rank=rank, world=world, engine_dtype=edt)
    sample_source = None
    if chief and not flags.synthetic and os.path.isdir(flags.sample_image_dir):
        sample_source = make_source(flags, B, shape, device, rank=0, world=1, data_dir=flags.sample_image_dir,
                                    seed_offset=99, shuffle_buffer=min(int(flags.shuffle_buffer), 4 * B),
                                    engine_dtype=edt)
    gen = torch.Generator().manual_seed(int(flags.seed) + 4242)
    sample_z = (torch.rand(B, cfg.z_dim, generator=gen) * 2 - 1).to(device)  # fixed (image_train.py:77)

    n_ex = source.num_examples
    if flags.train_size != math.inf:
        n_ex = min(n_ex, int(flags.train_size))
    step_per_epoch = max(1, -(-n_ex // (B * world)))
    max_steps = int(flags.max_steps)
    if flags.epoch and int(flags.epoch) > 0:
        max_steps = min(max_steps, int(flags.epoch) * step_per_epoch)

    writer = SummaryWriter(flags.checkpoint_dir) if (chief and flags.summaries) else None
    prof_range = None
    if flags.profile_steps:
        a, b = flags.profile_steps.split(":")
        prof_range = (int(a), int(b))
    prof = None
    fault_at = int(os.environ.get("DCGAN_FAULT_AT_STEP", "-1"))  # fault injection
    if os.environ.get("DCGAN_FAULT_RANK", "") not in ("", str(rank)):
        fault_at = -1

    step = int(engine.global_step)
    start_time = time.time()
    next_summary = start_time + float(flags.save_summaries_secs)
    last_rate_t, last_rate_step = start_time, step
    losslog = AsyncLossLog(engine, device)

    def emit(entries):
        for (st, t, ips), L in entries:
            print(STEP_LINE % (st // step_per_epoch, st % step_per_epoch, t, L["d_loss"], L["g_loss"]) +
                  ", images/sec: %.1f" % ips, file=out, flush=True)

    try:
        while step < max_steps:
            if prof_range and step == prof_range[0] and prof is None:
                prof = torch.profiler.profile(record_shapes=False, with_stack=False)
                prof.__enter__()
            engine.set_batch(source.next())
            engine.train_step()
            step += 1
            if prof is not None and step >= prof_range[1]:
                prof.__exit__(None, None, None)
                if chief:
                    prof.export_chrome_trace(os.path.join(flags.checkpoint_dir, "trace_rank%d.json" % rank))
                prof = None
            now = time.time()
            summary_due = chief and writer is not None and now >= next_summary
            if step % max(1, int(flags.log_every)) == 0 or summary_due or step == max_steps:
                ips = B * world * (step - last_rate_step) / max(1e-9, now - last_rate_t) if step > last_rate_step else 0.0
                losslog.push((step, now - start_time, ips))
                emit(losslog.ready(flush=summary_due or step == max_steps or bool(flags.timing)))
                if flags.timing and hasattr(engine, "phase_times"):
                    print("phase ms: " + ", ".join("%s %.3f" % kv for kv in engine.phase_times().items()),
                          file=out, flush=True)
                if summary_due:
                    L = engine.last_losses()
                    print("Running Summary operation on the chief.", file=out)
                    rate = (step - last_rate_step) / max(1e-9, now - last_rate_t)
                    vals = SUM.collect(engine, L, steps_per_sec=rate, loader_stats=source.stats())
                    writer.add_summary_values(vals, step)
                    writer.flush()
                    print("Finished running Summary operation.", file=out)
                    period = float(flags.save_summaries_secs)
                    next_summary = next_summary + period if period > 0 else now
                    while period > 0 and next_summary < now:
                        next_summary += period
                last_rate_t, last_rate_step = now, step
            sample_now = int(flags.sample_every) > 0 and step % int(flags.sample_every) == 1
            # the chief's time-based save decision is shared every SYNC_EVERY steps so that all
            # ranks take part in the BN moving-average averaging that precedes a save
            save_now = False
            if step % SYNC_EVERY == 0 or step == max_steps:
                due = chief and ckpt.save_secs > 0 and time.time() - ckpt.last_save >= ckpt.save_secs
                save_now = D.any_rank(due, device) if world > 1 else due
            if world > 1 and (sample_now or save_now):
                engine.sync_bn_state()
            if chief and sample_now:
                _sample(engine, flags, sample_source, source, sample_z, step, step_per_epoch, out)
            if chief and save_now:
                ckpt.save(engine)
            if int(flags.check_sync_every) > 0 and world > 1 and step % int(flags.check_sync_every) == 0:
                tens = (engine.sync_check_tensors() if hasattr(engine, "sync_check_tensors")
                        else [engine.model.g.flat, engine.model.d.flat])
                if not D.params_in_sync(tens, device):
                    raise RuntimeError("DDP divergence: parameters differ across ranks at step %d" % step)
            if fault_at >= 0 and step == fault_at:
                emit(losslog.ready(flush=True))  # the last step lines before a crash are the useful ones
                print("DCGAN_FAULT_AT_STEP=%d: simulated failure" % fault_at, file=out, flush=True)
                out.flush()
                os._exit(3)
        emit(losslog.ready(flush=True))
        if world > 1:
            engine.sync_bn_state()
        if chief:
            path = ckpt.save(engine)
            print("saved %s" % path, file=out)
    finally:
        try:  # pending step lines (a no-op after the normal flush above; kept on any exception)
            emit(losslog.ready(flush=True))
        except Exception:  # pragma: no cover - a dead device must not mask the original error
            pass
        source.close()
        if sample_source is not None:
            sample_source.close()
        if writer is not None:
            writer.close()
        D.barrier()
        D.shutdown()
    return 0


def _test_mode(engine, flags, cfg, B, device, info, chief, out) -> int:
    """``--nois_train``: sample-only mode (the flag the reference defines but never reads,
    ``image_train.py:23``). Restores the newest checkpoint, writes ``num_samples`` images from
    the EMA-BN sampler as grids, and with ``--visualize`` per-dimension z sweeps and a z
    interpolation (carpedm20-style DCGAN visualisations)."""
    if not info:
        raise SystemExit(" [!] no checkpoint in %s: train a model first, then run with --nois_train"
                         % flags.checkpoint_dir)
    if not chief:
        return 0
    gen = torch.Generator().manual_seed(int(flags.seed) + 31337)
    step = int(engine.global_step)
    n = max(1, int(flags.num_samples))
    imgs = []
    while sum(x.shape[0] for x in imgs) < n:
        z = (torch.rand(B, cfg.z_dim, generator=gen) * 2 - 1).to(device)
        imgs.append(engine.sampler(z).detach().float().cpu().numpy())
    arr = np.concatenate(imgs, 0)[:n]
    path = os.path.join(flags.sample_dir, "test_%06d.png" % step)
    IM.save_images(arr, (8, 8) if n == 64 else IM.grid_size(n), path)
    print("[Test] wrote %d samples to %s" % (n, path), file=out, flush=True)
    if flags.visualize:
        base = (torch.rand(1, cfg.z_dim, generator=gen) * 2 - 1).repeat(B, 1)
        sweep = torch.linspace(-1.0, 1.0, B)
        for d in range(min(cfg.z_dim, 8)):
            z = base.clone()
            z[:, d] = sweep
            x = engine.sampler(z.to(device)).detach().float().cpu().numpy()
            IM.save_images(x, IM.grid_size(B), os.path.join(flags.sample_dir, "test_arange_%d.png" % d))
        z0 = torch.rand(1, cfg.z_dim, generator=gen) * 2 - 1
        z1 = torch.rand(1, cfg.z_dim, generator=gen) * 2 - 1
        t = torch.linspace(0.0, 1.0, B).unsqueeze(1)
        x = engine.sampler(((1 - t) * z0 + t * z1).to(device)).detach().float().cpu().numpy()
        IM.save_images(x, IM.grid_size(B), os.path.join(flags.sample_dir, "test_interp.png"))
        print("[Visualize] wrote z sweeps and interpolation to %s" % flags.sample_dir, file=out, flush=True)
    return 0


def _sample(engine, flags, sample_source, source, sample_z, step, step_per_epoch, out) -> None:
    """Chief sampling side path (image_train.py:179-192): EMA-BN sampler grid + sample losses."""
    batch = (sample_source or source).next()
    samples = engine.sampler(sample_z)
    losses = engine.eval_losses(batch, sample_z)
    n = samples.shape[0]
    grid = (8, 8) if n == 64 else IM.grid_size(n)
    path = os.path.join(flags.sample_dir, "train_{:02d}_{:04d}.png".format(step // step_per_epoch,
                                                                          step % step_per_epoch))
    IM.save_images(samples.detach().float().cpu().numpy(), grid, path)
    print("[Sample] d_loss: %.8f, g_loss: %.8f" % (losses["d_loss"], losses["g_loss"]), file=out, flush=True)
