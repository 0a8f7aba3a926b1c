"""DDP path of the HIP engine on ONE GPU: two ranks share the card over the gloo backend
(RCCL refuses two ranks per GPU; the collective calls, streams, segmented hipGraphs and the
1/W gradient scale folded into Adam are the same code the RCCL run uses).

With identical data and rank-independent z on both ranks, the averaged gradient equals the
local one exactly (x + x = 2x, times 1/2 is exact in fp32), so W=2 must reproduce the
single-process engine BIT FOR BIT after several steps -- with graphs and without."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B = 16
STEPS = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(world, rank, graph):
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    cfg = DCGANConfig(output_size=64, c_dim=3)
    dev = torch.device("cuda", 0)
    eng = HipEngine(cfg, B, dev, seed=3, rank=rank, world=world, graph=graph, rank_seeded_z=False)
    real = torch.rand(B, 64, 64, 3, generator=torch.Generator().manual_seed(5)) * 2 - 1
    eng.set_batch(real.to(dev))
    return eng


def _run(eng):
    for _ in range(STEPS):
        eng.train_step()
    torch.cuda.synchronize()
    eng.gather_sharded_state()  # (collective; sharded update: every rank's conv-kernel shards)
    return eng.model.d.flat.cpu(), eng.model.g.flat.cpu(), eng.global_step


def _worker(rank, world, port, graph, out_dir, schedule="concurrent"):
    if schedule == "serial":
        os.environ["DCGAN_SERIAL_DBWD"] = "1"
    if schedule == "ddp":
        os.environ["DCGAN_DDP_SCHEDULE"] = "ddp"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DCGAN_DIST_BACKEND"] = "gloo"
    torch.cuda.set_device(0)
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    D.init_distributed(world, rank, torch.device("cuda", 0))
    eng = _make(world, rank, graph)
    d, g, step = _run(eng)
    assert eng._schedule() == schedule
    torch.save({"d": d, "g": g, "step": step, "graph": eng.graph_enabled}, os.path.join(out_dir, "r%d.pt" % rank))
    D.barrier()
    D.shutdown()


@pytest.mark.parametrize("graph,schedule", [(False, "concurrent"), (True, "concurrent"), (True, "serial"),
                                            (False, "ddp")])
def test_hip_ddp_two_ranks_match_single_process(tmp_path, graph, schedule):
    """The DDP schedules over two ranks: "concurrent" (D chain and G chain on separate streams,
    8 graph segments, collectives issued from both chains), "serial" (DCGAN_SERIAL_DBWD=1) and
    "ddp" (the one-graph RCCL schedule with per-layer G buckets, run eagerly under gloo)."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, graph, str(tmp_path), schedule)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r0["graph"] == (graph and schedule != "ddp")
    assert torch.equal(r0["d"], r1["d"]) and torch.equal(r0["g"], r1["g"])
    assert r0["step"] == STEPS
    eng = _make(1, 0, graph)
    d, g, _ = _run(eng)
    assert torch.equal(r0["d"], d), (r0["d"] - d).abs().max()
    assert torch.equal(r0["g"], g), (r0["g"] - g).abs().max()


def _shard_worker(rank, world, port, out_dir, shard):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DCGAN_DIST_BACKEND"] = "gloo"
    os.environ["DCGAN_DDP_SHARD"] = shard
    torch.cuda.set_device(0)
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    D.init_distributed(world, rank, torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    eng = HipEngine(DCGANConfig(output_size=64, c_dim=3), B, dev, seed=3, rank=rank, world=world, graph=False)
    assert eng._sharded() == (shard == "1") and eng._schedule() == "concurrent"
    for s in range(STEPS):  # rank-specific batches and z
        eng.set_batch((torch.rand(B, 64, 64, 3, generator=torch.Generator().manual_seed(100 + 7 * s + rank)) * 2
                       - 1).to(dev))
        eng.train_step()
    torch.cuda.synchronize()
    mirrors = (eng.wbf_d.flat.cpu().clone(), eng.wbf_g.flat.cpu().clone())
    eng.sync_bn_state()  # what the trainer runs before a checkpoint: gathers the sharded state
    torch.save({"d": eng.model.d.flat.cpu(), "g": eng.model.g.flat.cpu(), "md": eng.opt_d.m.flat.cpu(),
                "vg": eng.opt_g.v.flat.cpu(), "wd": mirrors[0], "wg": mirrors[1], "pd": eng.opt_d.powers.cpu(),
                "step": eng.global_step, "L": eng.last_losses()}, os.path.join(out_dir, "s%s_%d.pt" % (shard, rank)))
    D.barrier()
    D.shutdown()


def test_sharded_update_matches_allreduce_two_ranks(tmp_path):
    """DDP default (eager segmented step, bf16): reduce-scatter the conv kernels' gradients, Adam
    on this rank's half, all-gather the bf16 mirror. With DIFFERENT batches per rank, after 4 steps
    and the pre-checkpoint gather, masters / Adam slots / mirrors / powers / losses equal the
    all-reduce step's bit for bit (a two-rank fp32 sum is exact in either order), on both ranks;
    before the gather the mirrors already agree."""
    ctx = mp.get_context("spawn")
    res = {}
    for shard in ("1", "0"):
        port = _free_port()
        procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, str(tmp_path), shard)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=600)
            assert p.exitcode == 0, "rank exited with %s" % p.exitcode
        res[shard] = [torch.load(tmp_path / ("s%s_%d.pt" % (shard, r)), weights_only=True) for r in range(2)]
    ref = res["0"][0]
    for r in res["1"] + res["0"][1:]:
        for k in ("d", "g", "md", "vg", "wd", "wg", "pd"):
            assert torch.equal(r[k], ref[k]), (k, (r[k].float() - ref[k].float()).abs().max())
        assert r["step"] == STEPS
    for rank in range(2):  # the losses are rank-local (each rank's own batch)
        assert res["1"][rank]["L"] == res["0"][rank]["L"], rank


def _real(rank):
    return torch.rand(B, 64, 64, 3, generator=torch.Generator().manual_seed(100 + rank)) * 2 - 1


def _one_step_grads(world, rank, graph):
    """One training step with rank-specific data and rank-seeded z; returns the gradient buffers
    after the step (after the all-reduce at W > 1: the SUM over ranks, Adam applies the 1/W)."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    dev = torch.device("cuda", 0)
    eng = HipEngine(DCGANConfig(output_size=64, c_dim=3), B, dev, seed=3, rank=rank, world=world, graph=graph,
                    rank_seeded_z=True)
    eng.set_batch(_real(rank).to(dev))
    eng.train_step()
    torch.cuda.synchronize()
    return eng.grad_d.flat.cpu().clone(), eng.grad_g.flat.cpu().clone(), eng.model.d.flat.cpu(), eng.model.g.flat.cpu()


def _grad_worker(rank, world, port, graph, out_dir, schedule):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DCGAN_DIST_BACKEND"] = "gloo"
    os.environ["DCGAN_DDP_SCHEDULE"] = schedule
    torch.cuda.set_device(0)
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    D.init_distributed(world, rank, torch.device("cuda", 0))
    gd, gg, d, g = _one_step_grads(world, rank, graph)
    torch.save({"gd": gd, "gg": gg, "d": d, "g": g}, os.path.join(out_dir, "g%d.pt" % rank))
    D.barrier()
    D.shutdown()


@pytest.mark.parametrize("graph,schedule", [(True, "concurrent"), (False, "ddp")])
def test_hip_ddp_different_rank_batches_sum_gradients(tmp_path, graph, schedule):
    """Two ranks with DIFFERENT real batches and z: the all-reduced gradient in every slice (D's
    top layer + head, the rest of D, every G layer) equals the sum of the two single-process
    engines' gradients on the same per-rank inputs, bit for bit (a two-term fp32 sum is exact in
    either order), and both ranks hold the same weights after the update."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, graph, str(tmp_path), schedule)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
    r0 = torch.load(tmp_path / "g0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "g1.pt", weights_only=True)
    assert torch.equal(r0["d"], r1["d"]) and torch.equal(r0["g"], r1["g"])
    assert torch.equal(r0["gd"], r1["gd"]) and torch.equal(r0["gg"], r1["gg"])
    a = _one_step_grads(1, 0, graph)
    b = _one_step_grads(1, 1, graph)
    assert not torch.equal(a[0], b[0]) and not torch.equal(a[1], b[1]), "per-rank inputs must differ"
    assert torch.equal(r0["gd"], a[0] + b[0]), (r0["gd"] - (a[0] + b[0])).abs().max()
    assert torch.equal(r0["gg"], a[1] + b[1]), (r0["gg"] - (a[1] + b[1])).abs().max()


WIRE_STEPS = 50


def _wire_run(world, rank, wire, noise_seed=None):
    """WIRE_STEPS steps of the DDP engine (rank-independent data and z) with the given all-reduce
    wire dtype; noise_seed: 4e-3 relative noise on the first batch (the envelope runs)."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    dev = torch.device("cuda", 0)
    eng = HipEngine(DCGANConfig(output_size=64, c_dim=3), B, dev, seed=11, rank=rank, world=world, graph=True,
                    rank_seeded_z=False, allreduce_dtype=wire)
    gen = torch.Generator().manual_seed(9)
    losses = []
    for s in range(WIRE_STEPS):
        real = (torch.rand(B, 64, 64, 3, generator=gen) * 2 - 1).to(dev)
        if s == 0 and noise_seed is not None:
            real = real * (1 + 4e-3 * torch.randn(real.shape, generator=torch.Generator().manual_seed(noise_seed)).to(dev))
        eng.set_batch(real)
        eng.train_step()
        losses.append([eng.last_losses()[k] for k in ("d_loss", "g_loss")])
    torch.cuda.synchronize()
    return torch.tensor(losses, dtype=torch.float64), eng.model.g.flat.cpu(), eng.model.d.flat.cpu()


def _wire_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DCGAN_DIST_BACKEND"] = "gloo"
    torch.cuda.set_device(0)
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    D.init_distributed(world, rank, torch.device("cuda", 0))
    L, g, d = _wire_run(world, rank, "bf16")
    torch.save({"L": L, "g": g, "d": d}, os.path.join(out_dir, "w%d.pt" % rank))
    D.barrier()
    D.shutdown()


def test_bf16_wire_holds_the_50_step_envelope(tmp_path):
    """--allreduce_dtype bf16 (half the wire bytes) over two ranks with rank-independent inputs:
    the averaged gradient is the bf16-rounded local one, so the run may drift from the exact
    (fp32-wire) single-process run only as far as a bf16-sized perturbation of that run does:
    steps 0-1 within 5 % (+0.05), mean |d_loss| / |g_loss| deviation over steps 10-49 within 2.5x
    the envelope's (+0.05), ranks identical, every loss finite."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_wire_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=900)
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
    r0 = torch.load(tmp_path / "w0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "w1.pt", weights_only=True)
    assert torch.equal(r0["g"], r1["g"]) and torch.equal(r0["d"], r1["d"])
    L = r0["L"]
    assert torch.isfinite(L).all()
    ref, _, _ = _wire_run(1, 0, "fp32")
    envs = [_wire_run(1, 0, "fp32", noise_seed=13 + i)[0] for i in range(2)]
    early = (L[:2] - ref[:2]).abs() > 0.05 * ref[:2].abs() + 0.05
    assert not early.any(), (L[:2], ref[:2])
    dev = (L[10:] - ref[10:]).abs().mean(0)
    env = torch.maximum(*[(e[10:] - ref[10:]).abs().mean(0) for e in envs])
    print("\nbf16 wire vs exact over %d steps: mean |dev| d_loss %.3f g_loss %.3f; envelope %.3f %.3f"
          % (WIRE_STEPS, dev[0], dev[1], env[0], env[1]))
    assert (dev <= 2.5 * env + 0.05).all(), (dev, env)


def test_timed_concurrent_schedule_matches_fused():
    """The per-phase timed step (8 concurrent graph segments incl. G_tail and adam_G_a, the DDP schedule at W=1)
    is the same computation as the single fused graph, bit for bit; phase ends are reported."""
    a = _make(1, 0, True)
    b = _make(1, 0, True)
    b.enable_timing()
    assert a._schedule() == "fused" and b._schedule() == "concurrent"
    d0, g0, _ = _run(a)
    d1, g1, _ = _run(b)
    assert torch.equal(d0, d1) and torch.equal(g0, g1)
    pt = b.phase_times()
    assert set(pt) == {"fwd@end", "D_bwd_top@end", "G_chain@end", "D_bwd_rest@end", "G_tail@end", "adam_G_a@end",
                       "adam_G@end", "adam_D@end"}
    assert all(v > 0 for v in pt.values())


def test_bench_two_ranks_json_contract(tmp_path):
    """bench.py's multi-rank path (torch.distributed.run, barrier + sync bracketing, MAX over
    ranks, one JSON line from rank 0) with two ranks on this one GPU over gloo -- the driver's
    N>1 scaling runs take the same code with RCCL, one rank per GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DCGAN_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "2",
           "--steps", "4", "--warmup", "2"]
    out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 4 and res["warmup"] == 2
    assert res["config"]["global_batch"] == 256 and res["config"]["parallelism"] == "dp2"
    assert res["value"] > 0 and res["higher_is_better"] is True and res["scaling"] == "weak"


def test_bench_direct_two_ranks_self_launch(tmp_path):
    """``python bench.py --gpus 2`` with NO outer launcher (the driver's own command form):
    bench.py starts the two ranks itself (child processes, the parent never touches the GPU).
    gloo lets both ranks share this one GPU; on an 8-GPU node the same path runs RCCL."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DCGAN_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2"]
    out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "[launch]" not in out.stdout, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["world_size"] == 2 and len(res["config"]["devices"]) == 2
    assert res["config"]["backend"] == "gloo" and res["value"] > 0


def _rccl_worker(out_dir, graph, port, schedule):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DCGAN_FORCE_DDP"] = "1"
    os.environ["DCGAN_DDP_SCHEDULE"] = schedule
    os.environ.pop("DCGAN_DIST_BACKEND", None)
    torch.cuda.set_device(0)
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    import torch.distributed as tdist
    D.init_distributed(1, 0, torch.device("cuda", 0))
    eng = _make(1, 0, graph)
    assert eng.ddp and eng._schedule() == schedule
    assert eng._ddp_gw_alt() == (schedule == "concurrent" and not graph)
    d, g, step = _run(eng)
    torch.save({"d": d, "g": g, "step": step, "backend": tdist.get_backend(), "world": tdist.get_world_size(),
                "graph": eng.graph_enabled, "graphs": len(eng._graphs)}, os.path.join(out_dir, "rccl.pt"))
    D.barrier()
    D.shutdown()


@pytest.mark.parametrize("graph,schedule", [(False, "ddp"), (True, "ddp"), (True, "concurrent"), (False, "concurrent")])
def test_rccl_single_rank_ddp_matches_fused(tmp_path, graph, schedule):
    """The REAL collective path on a one-GPU box: a one-rank RCCL (backend "nccl") process group
    (DCGAN_FORCE_DDP=1). "ddp": the RCCL all-reduces captured INSIDE the step's single hipGraph
    (per-layer G buckets); "concurrent": issued on the comm stream between 8 segments (graphs or
    eager replay; eager: G's weight gradients on alt1). All
    bit-identical to the fused single-graph step."""
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_rccl_worker, args=(str(tmp_path), graph, _free_port(), schedule))
    p.start()
    p.join(timeout=600)
    assert p.exitcode == 0, "RCCL rank exited with %s" % p.exitcode
    r = torch.load(tmp_path / "rccl.pt", weights_only=True)
    assert r["backend"] == "nccl" and r["world"] == 1 and r["step"] == STEPS and r["graph"] == graph
    if graph:
        assert r["graphs"] == (1 if schedule == "ddp" else 8)
    eng = _make(1, 0, True)
    assert not eng.ddp and eng._schedule() == "fused"
    d, g, _ = _run(eng)
    assert torch.equal(r["d"], d), (r["d"] - d).abs().max()
    assert torch.equal(r["g"], g), (r["g"] - g).abs().max()


def test_bench_force_ddp_reports_rccl():
    """bench.py --force_ddp at N=1: the timed step runs the DDP path over a one-rank RCCL group
    and the JSON line says so (backend nccl, world_size 1)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("DCGAN_DIST_BACKEND", None)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "5", "--warmup", "2",
                          "--force_ddp", "--graph", "1"], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert res["config"]["backend"] == "nccl" and res["config"]["world_size"] == 1
    assert res["config"]["collectives"] == "torch.distributed(nccl)"
    assert res["config"]["schedule"] == "concurrent" and res["config"]["graphs_per_step"] == 8
    assert res["n_gpus"] == 1 and res["value"] > 0


def _wire_copyfree_worker(out_dir, port, schedule):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DCGAN_FORCE_DDP"] = "1"
    os.environ["DCGAN_DDP_SCHEDULE"] = schedule
    os.environ.pop("DCGAN_DIST_BACKEND", None)
    torch.cuda.set_device(0)
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    D.init_distributed(1, 0, torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    eng = HipEngine(DCGANConfig(output_size=64, c_dim=3), B, dev, seed=3, graph=True, rank_seeded_z=False,
                    allreduce_dtype="bf16")
    assert eng._schedule() == schedule and eng._wire_direct() == (schedule == "concurrent")
    real = torch.rand(B, 64, 64, 3, generator=torch.Generator().manual_seed(5)) * 2 - 1
    eng.set_batch(real.to(dev))
    d, g, _ = _run(eng)
    torch.save({"d": d, "g": g}, os.path.join(out_dir, "wire_%s.pt" % schedule))
    D.barrier()
    D.shutdown()


def test_bf16_wire_without_copies_matches_the_copying_reducer(tmp_path):
    """The segmented step's copy-free bf16 wire (cast kernels inside the step graphs, RCCL reducing
    the bf16 images in place, Adam reading them) gives bit for bit the weights of the reducer's
    fp32 -> bf16 -> fp32 copying path (serial schedule), over a one-rank RCCL group."""
    ctx = mp.get_context("spawn")
    for sch in ("concurrent", "serial"):
        p = ctx.Process(target=_wire_copyfree_worker, args=(str(tmp_path), _free_port(), sch))
        p.start()
        p.join(timeout=600)
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
    a = torch.load(tmp_path / "wire_concurrent.pt", weights_only=True)
    b = torch.load(tmp_path / "wire_serial.pt", weights_only=True)
    assert torch.equal(a["d"], b["d"]), (a["d"] - b["d"]).abs().max()
    assert torch.equal(a["g"], b["g"]), (a["g"] - b["g"]).abs().max()


def _native_worker(out_dir, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.pop("DCGAN_DIST_BACKEND", None)
    torch.cuda.set_device(0)
    from distributed_tensorflow_for_dcgan_amd.ops import hip as H
    from distributed_tensorflow_for_dcgan_amd.parallel import dist as D
    D.init_distributed(1, 0, torch.device("cuda", 0), force=True)
    comm = D.native_comm(torch.device("cuda", 0))
    assert comm is not None and comm.nranks == 1 and comm.rank == 0
    x = torch.randn(3000, device="cuda")
    ref = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    comm.all_reduce(x.data_ptr(), x.numel(), 0, s.cuda_stream)  # one rank: the sum is the input
    torch.cuda.current_stream().wait_stream(s)
    ok1 = torch.equal(x, ref)
    y = torch.randn(4096, device="cuda").to(torch.bfloat16)
    yref = y.clone()
    prog = H.ext().Program()
    prog.allreduce("ar", comm, y.data_ptr(), y.numel(), 1, 0)
    g = torch.cuda.CUDAGraph()  # the recorded collective is graph-capturable
    with torch.cuda.graph(g):
        H.run(prog)
    g.replay()
    torch.cuda.synchronize()
    torch.save({"ok1": ok1, "ok2": torch.equal(y, yref)}, os.path.join(out_dir, "native.pt"))
    D.shutdown()


def test_native_rccl_communicator():
    """The engine's native RCCL communicator (csrc/comm.h: PyTorch's librccl via dlopen, our own
    ncclComm from a broadcast unique id): ncclAllReduce on a given stream, and as a recorded
    Program op inside a captured hipGraph, over a one-rank group."""
    import tempfile
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        p = ctx.Process(target=_native_worker, args=(d, _free_port()))
        p.start()
        p.join(timeout=300)
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
        r = torch.load(os.path.join(d, "native.pt"), weights_only=True)
    assert r["ok1"] and r["ok2"]
