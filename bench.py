#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node), 64x64x3 DCGAN, bs=128 per GPU.

``python bench.py --gpus N --steps K --warmup W`` runs the full reference-semantics
DCGAN training step (G fwd, D(real)+D(fake) fwd, 3 losses, D/G backward, gradient
all-reduce over RCCL when N>1, two TF-Adam updates) on synthetic images of the BASELINE
shape with random-init weights. For N>1 it runs one rank per GPU: either under
``torch.distributed.run`` (WORLD_SIZE set) or, when started directly, by launching N child
ranks itself (``self_launch``). W untimed warmup steps, then EXACTLY K timed steps between a
barrier + device sync on both sides; the per-rank time is MAX-reduced over ranks and
rank 0 prints one JSON line. ``value`` = N * batch * K / max_time (weak scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_VALUE = None  # the reference publishes no number ("published": {})


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch_size", type=int, default=128, help="per-GPU batch")
    p.add_argument("--output_size", type=int, default=64)
    p.add_argument("--c_dim", type=int, default=3)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    p.add_argument("--engine", default="hip", choices=["hip", "reference"])
    # eager C++ replay of the recorded Programs (0) measured 1.1-1.5 % faster than hipGraph replay (1)
    # for the fused step and 3 % for the segmented DDP step (profiles/r5/ab_eager_vs_graph_r5.txt)
    p.add_argument("--graph", type=int, default=0, help="1: replay the step as hipGraph(s) (hip engine); 0: C++ replay")
    p.add_argument("--allreduce_dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--force_ddp", action="store_true",
                   help="run the data-parallel step (process group + RCCL collectives) even at N=1")
    return p.parse_args()


def self_launch(args) -> int:
    """``python bench.py --gpus N`` (N > 1) without an outer launcher: start N child ranks, one
    per GPU, with the torch.distributed.run env contract (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_*; rendezvous on 127.0.0.1). The parent never touches a GPU (it only COUNTS devices,
    which initialises no HIP context) and never exec()s: it waits for the children, stops the
    rest when one fails, and returns the worst exit code. Rank 0's JSON line reaches stdout
    directly (the children inherit it); launcher messages go to stderr. The N-worker reference
    starts one process per task by hand (``/root/reference/image_train.py:52-67``)."""
    from distributed_tensorflow_for_dcgan_amd.launch import launch
    gloo = os.environ.get("DCGAN_DIST_BACKEND", "") == "gloo"
    n_dev = torch.cuda.device_count()
    if n_dev < args.gpus and not gloo:
        # (DCGAN_DIST_BACKEND=gloo: rehearsal, ranks may share a GPU or run on the CPU)
        print("bench.py: --gpus %d but only %d GPU(s) visible" % (args.gpus, n_dev), file=sys.stderr)
        return 2
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    return launch(args.gpus, cmd, max_restarts=0, master_addr="127.0.0.1",
                  log=lambda m: print(m, file=sys.stderr, flush=True))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if rank == 0:
            print("bench.py: --gpus %d but WORLD_SIZE=%d (launch with torch.distributed.run)" % (args.gpus, world),
                  file=sys.stderr)
        sys.exit(2)

    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    from distributed_tensorflow_for_dcgan_amd.engine.factory import build_engine

    # (local_rank modulo the visible GPUs only matters for the 1-GPU rehearsal of the multi-rank
    # path over gloo, DCGAN_DIST_BACKEND=gloo; one rank per GPU otherwise)
    device = (torch.device("cuda", local_rank % max(1, torch.cuda.device_count())) if torch.cuda.is_available()
              else torch.device("cpu"))
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if args.force_ddp:
        os.environ["DCGAN_FORCE_DDP"] = "1"
    pg = D.init_distributed(world, rank, device)
    cfg = DCGANConfig(output_size=args.output_size, c_dim=args.c_dim)
    eng = build_engine(cfg, args.batch_size, device, engine=args.engine, dtype=args.dtype, seed=args.seed,
                       rank=rank, world=world, graph=bool(args.graph), allreduce_dtype=args.allreduce_dtype)
    gen = torch.Generator(device="cpu").manual_seed(args.seed + 1000 * rank)
    real = (torch.rand(args.batch_size, cfg.output_size, cfg.output_size, cfg.c_dim, generator=gen) * 2 - 1)
    real = real.to(device)
    eng.set_synthetic_batch(real)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        eng.train_step()
    sync()
    D.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.train_step()
    sync()
    D.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = D.max_over_ranks(dt, device)
    losses = eng.last_losses()
    # self-verifying multi-GPU record: which backend the process group used, how many ranks it
    # saw, and every rank's HIP device (all-gathered), so "RCCL saw N distinct GPUs" is checkable
    backend, world_seen, devices = "none", 1, [torch.cuda.current_device() if device.type == "cuda" else -1]
    if D.is_initialized():
        import torch.distributed as tdist
        backend, world_seen = tdist.get_backend(), tdist.get_world_size()
        mine = torch.tensor([devices[0]], dtype=torch.int64, device=device if backend == "nccl" else "cpu")
        allv = [torch.zeros_like(mine) for _ in range(world_seen)]
        tdist.all_gather(allv, mine)
        devices = [int(v.item()) for v in allv]
    imgs = args.gpus * args.batch_size * args.steps
    value = imgs / dt
    ms = dt / args.steps * 1e3
    if rank == 0:
        res = {
            "metric": ("images/sec (whole node), 64x64 DCGAN bs=128/GPU at 1/2/4/8 MI355X"
                       if (cfg.output_size, cfg.c_dim, args.batch_size) == (64, 3, 128)
                       else "images/sec (whole node), %dx%dx%d DCGAN bs=%d/GPU"
                       % (cfg.output_size, cfg.output_size, cfg.c_dim, args.batch_size)),
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": getattr(eng, "dtype_name", args.dtype),
            "data": "synthetic (uniform[-1,1] images of shape [B,%d,%d,%d]; random-init weights)"
                    % (cfg.output_size, cfg.output_size, cfg.c_dim),
            "config": {"model": "DCGAN-{0}x{0}x{1} (G {2:,} / D {3:,} params)".format(
                           cfg.output_size, cfg.c_dim, cfg.param_counts()["g"], cfg.param_counts()["d"]),
                       "global_batch": args.batch_size * args.gpus, "per_gpu_batch": args.batch_size,
                       "seq_len": None, "parallelism": "dp%d" % args.gpus, "engine": eng.name,
                       "hip_graph": bool(getattr(eng, "graph_enabled", False)),
                       "schedule": eng._schedule() if hasattr(eng, "_schedule") else None,
                       "graphs_per_step": sum(g is not None for g in getattr(eng, "_graphs", [])) or None,
                       "backend": backend, "world_size": world_seen, "devices": devices,
                       "collectives": getattr(eng, "comm_kind", None),
                       "kernels_per_step": eng.kernel_count() if hasattr(eng, "kernel_count") else None,
                       "gflop_per_image": round(cfg.flops_per_image() / 1e9, 4),
                       "tflops_achieved": round(value * cfg.flops_per_image() / 1e12, 2),
                       "last_losses": {k: round(float(v), 5) for k, v in losses.items()}},
        }
        print(json.dumps(res), flush=True)
    D.shutdown()


if __name__ == "__main__":
    main()
