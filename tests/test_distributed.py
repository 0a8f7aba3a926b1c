"""Synchronous data parallelism on CPU with the gloo backend (world_size 2).

The RCCL (backend "nccl") path is the same code with GPU tensors; it runs at round end on an
8-GPU node. Here: gradient averaging == manual mean of per-rank gradients, parameters stay
bit-identical across ranks, bucketed all-reduce, the multi-process CLI."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker_ddp(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    from distributed_tensorflow_for_dcgan_amd.engine.factory import ReferenceEngine
    from distributed_tensorflow_for_dcgan_amd.engine.reference_step import ReferenceStep
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    from distributed_tensorflow_for_dcgan_amd.models.dcgan import DCGAN
    from distributed_tensorflow_for_dcgan_amd.ops import reference as R
    dev = torch.device("cpu")
    D.init_distributed(world, rank, dev)
    cfg = DCGANConfig(output_size=28, c_dim=1)
    eng = ReferenceEngine(cfg, 4, dev, seed=rank * 100, rank=rank, world=world)  # different seeds: bcast fixes
    real = torch.rand(4, 28, 28, 1, generator=torch.Generator().manual_seed(10 + rank)) * 2 - 1
    eng.set_batch(real)
    # expected update: mean over ranks of the local gradients at the broadcast init
    probe = DCGAN(cfg, device=dev)
    probe.g.flat.copy_(eng.model.g.flat)
    probe.d.flat.copy_(eng.model.d.flat)
    zgen_state = eng.z_gen.get_state()
    z = torch.rand(4, cfg.z_dim, generator=eng.z_gen) * 2 - 1
    eng.z_gen.set_state(zgen_state)
    _, gd, gg = ReferenceStep(probe).compute_grads(real, z, update_ema=False)
    dist.all_reduce(gd)
    dist.all_reduce(gg)
    gd /= world
    gg /= world
    exp_d, exp_g = probe.d.flat.clone(), probe.g.flat.clone()
    for w, g in ((exp_d, gd), (exp_g, gg)):
        m, v = torch.zeros_like(w), torch.zeros_like(w)
        R.tf_adam_update(w, g, m, v, 0.5, 0.999, 2e-4, 0.5)
    eng.train_step()
    ok_update = torch.allclose(eng.model.d.flat, exp_d, atol=1e-6) and torch.allclose(eng.model.g.flat, exp_g,
                                                                                       atol=1e-6)
    flats = [torch.zeros_like(eng.model.g.flat) for _ in range(world)]
    dist.all_gather(flats, eng.model.g.flat)
    same = all(torch.equal(flats[0], f) for f in flats)
    # bucketed all-reduce of a flat buffer
    buf = torch.arange(1000, dtype=torch.float32) * (rank + 1)
    ar = D.GradAllReducer(buf, bucket_mb=0.001)
    assert len(ar.buckets) > 1
    ar.launch()
    ar.wait()
    ok_ar = torch.allclose(buf, torch.arange(1000, dtype=torch.float32) * 1.5)
    flag = D.any_rank(rank == 1, dev)
    # divergence detector: in sync now; a one-ulp change on one rank is caught
    sync_ok = D.params_in_sync([eng.model.g.flat, eng.model.d.flat], dev)
    if rank == 1:
        eng.model.d.flat[7] = torch.nextafter(eng.model.d.flat[7], torch.tensor(1.0))
    sync_bad = D.params_in_sync([eng.model.g.flat, eng.model.d.flat], dev)
    if rank == 0:
        torch.save({"update": ok_update, "same": same, "ar": ok_ar, "any": flag, "sync": sync_ok and not sync_bad},
                   out_path)
    D.shutdown()


def test_ddp_gloo_two_ranks(tmp_path):
    out = str(tmp_path / "res.pt")
    mp.spawn(_worker_ddp, args=(2, _free_port(), out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    assert res == {"update": True, "same": True, "ar": True, "any": True, "sync": True}


def test_cli_two_processes_gloo(tmp_path):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        cmd = [sys.executable, os.path.join(ROOT, "image_train.py"), "--synthetic", "--output_size=28", "--c_dim=1",
               "--batch_size=4", "--max_steps=3", "--device=cpu", "--checkpoint_dir=%s" % (tmp_path / "ck"),
               "--sample_dir=%s" % (tmp_path / "s"), "--save_summaries_secs=1000", "--sample_every=2",
               "--check_sync_every=1"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=600)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "Epoch: [ 0] step: [ 3]" in outs[0]
    assert os.path.exists(tmp_path / "ck" / "model.ckpt-3.index")
    assert os.path.exists(tmp_path / "s" / "train_00_0001.png")


def test_launcher_restarts_after_fault_and_resumes(tmp_path):
    """2 gloo ranks under the restart launcher: the chief dies at step 10 (fault injection,
    right after its checkpoint at step 10), the launcher stops rank 1 (blocked in the next
    collective), restarts both; they resume from step 10 and finish at step 14."""
    cmd = [sys.executable, "-m", "distributed_tensorflow_for_dcgan_amd.launch", "--nproc", "2", "--max_restarts", "2",
           "--grace", "5", "--", os.path.join(ROOT, "image_train.py"), "--synthetic", "--output_size=28",
           "--c_dim=1", "--batch_size=4", "--max_steps=14", "--device=cpu",
           "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "s"),
           "--save_summaries_secs=1000", "--sample_every=0", "--save_model_secs=1e-9"]
    env = dict(os.environ, OMP_NUM_THREADS="2", DCGAN_FAULT_AT_STEP="10", DCGAN_FAULT_RANK="0",
               PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900,
                       cwd=ROOT)
    assert p.returncode == 0, p.stdout
    assert "[launch] restart 1/2" in p.stdout
    assert "global_step 10" in p.stdout  # resumed
    assert os.path.exists(tmp_path / "ck" / "model.ckpt-14.index")


def test_reference_style_worker_hosts_launch(tmp_path):
    """The reference's own launch form (image_train.py:52-66): one process per worker, cluster
    given by --worker_hosts/--task_index, no torchrun environment. Both workers train together
    (gloo on CPU here) and worker 1 maps to local GPU index 1."""
    p0, p1 = _free_port(), _free_port()
    hosts = "127.0.0.1:%d,127.0.0.1:%d" % (p0, p1)
    procs = []
    for r in range(2):
        env = dict(os.environ, OMP_NUM_THREADS="2")
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        cmd = [sys.executable, os.path.join(ROOT, "image_train.py"), "--job_name=worker", "--task_index=%d" % r,
               "--worker_hosts=" + hosts, "--ps_hosts=127.0.0.1:%d" % _free_port(), "--synthetic",
               "--output_size=28", "--c_dim=1", "--batch_size=4", "--max_steps=2", "--device=cpu", "--verbose",
               "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "s"),
               "--save_summaries_secs=1000", "--sample_every=0", "--check_sync_every=1"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=600)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "rank 0/2 local_rank 0 (worker_hosts)" in outs[0]
    assert "rank 1/2 local_rank 1 (worker_hosts)" in outs[1]
    assert "Epoch: [ 0] step: [ 2]" in outs[0]


def _bench_env(**kw):
    env = dict(os.environ, OMP_NUM_THREADS="2", **kw)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DCGAN_DIST_BACKEND"):
        if k not in kw:
            env.pop(k, None)
    return env


def test_bench_refuses_more_ranks_than_gpus():
    """``python bench.py --gpus 2`` without an outer launcher and without 2 visible GPUs exits
    2 with a message naming the GPU count, before starting any rank."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=_bench_env(), capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 2
    assert "--gpus 2 but only 0 GPU(s) visible" in p.stderr
    assert p.stdout.strip() == ""


def test_bench_self_launches_ranks_gloo_cpu():
    """The driver's direct form ``python bench.py --gpus 2`` (no torch.distributed.run): bench.py
    starts two child ranks itself; here over gloo on the CPU with the reference engine. Rank 0
    prints exactly one JSON line on stdout (launcher messages go to stderr; gloo's own C++
    connection notices also land on stdout, RCCL prints none)."""
    import json
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--engine", "reference", "--dtype", "fp32", "--output_size", "28", "--c_dim", "1", "--batch_size", "4"]
    p = subprocess.run(cmd, env=_bench_env(DCGAN_DIST_BACKEND="gloo"), capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    assert "[launch]" not in p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["world_size"] == 2 and res["config"]["backend"] == "gloo"
    assert res["config"]["parallelism"] == "dp2" and res["config"]["global_batch"] == 8
    assert "[launch] all 2 ranks finished" in p.stderr
