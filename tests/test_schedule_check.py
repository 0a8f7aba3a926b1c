"""CPU tests of the stream-hazard checker (engine/schedule_check.py): every schedule of the HIP
engine, for every element type, single process and DDP, is free of unordered overlapping
accesses -- and the checker does find the round-1 race when it is re-introduced."""
import pytest
import torch

from distributed_tensorflow_for_dcgan_amd.engine import schedule_check as SC
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig

CASES = [(1, None, False), (1, None, True), (1, "serial", False), (2, None, False), (2, "ddp", False),
         (2, "serial", False)]


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("world,schedule,timing", CASES)
def test_schedule_has_no_stream_hazards(dtype, world, schedule, timing):
    sched, hz, n = SC.check(DCGANConfig(), 4, dtype, world, schedule, timing)
    expect = schedule or ("fused" if world == 1 and not timing else "concurrent")
    assert sched == expect
    assert n > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


@pytest.mark.parametrize("size", [28, 128])
def test_other_resolutions_have_no_stream_hazards(size):
    c = 1 if size == 28 else 3
    for world, schedule, timing in ((1, None, False), (2, None, False), (2, "ddp", False)):
        _, hz, _ = SC.check(DCGANConfig(output_size=size, c_dim=c), 2, "bf16", world, schedule, timing)
        assert hz == [], "\n".join(map(str, hz[:10]))


def _dry(world=1, timing=False, schedule=None):
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=world, dry_run=True, graph=False, schedule=schedule)
    if timing:
        eng._timing = True
        eng._build_updates()
    return eng


def test_checker_finds_the_round1_adam_race():
    """Round 1: at W=1 with --timing the concurrent schedule kept the fused two-model Adam in
    its first update segment, which ran before the main stream joined the D chain."""
    eng = _dry(timing=True)
    assert eng._schedule() == "concurrent"
    hz, _ = SC.check_engine(eng)
    assert hz == []
    eng.progC = eng._prog()
    eng._build_update_fused(eng.progC)   # the round-1 program
    eng._c_split = eng.progC.size()      # ... all of it in the first update segment

    def round1_order(ex):                # ... issued before the cs <- D-chain join
        cs, alt = ex.main(), ex.alt[0]
        ex.run(eng.progA, [cs, ex.side], 0, eng._a_fwd)
        ex.wait(alt, cs)
        ex.run(eng.progB, ex.alt)
        ex.run(eng.progA, [cs, ex.side], eng._a_fwd, -1)
        ex.run(eng.progW, [cs, ex.side])
        ex.run(eng.progC, [cs, ex.side], 0, eng._c_split)
        ex.wait(cs, alt)

    eng._run_step = round1_order
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed the Adam(D) / D-backward race"
    txt = "\n".join(map(str, hz))
    assert "adam_gd" in txt and "alt0" in txt


def test_checker_finds_a_missing_join():
    """Dropping the join of the D chain before the update is reported."""
    eng = _dry()

    def bad_fused(ex, cs):
        ex.run(eng.progA, [cs, ex.side], 0, eng._a_fwd)
        ex.wait(ex.alt[0], cs)
        ex.run(eng.progB, ex.alt)
        ex.run(eng.progA, [cs, ex.side], eng._a_fwd, -1)
        ex.run(eng.progC, [cs, ex.side])  # no ex.wait(cs, alt0)

    eng._run_fused = bad_fused
    hz, _ = SC.check_engine(eng)
    assert any("adam" in h.a or "adam" in h.b for h in hz)


def test_op_accesses_are_recorded():
    eng = _dry()
    names = set()
    for p in (eng.progA, eng.progB, eng.progW, eng.progC):
        for i in range(p.size()):
            name, slot, kind, ev, acc = p.op_info(i)
            names.add(name)
            if kind == eng.ext.OP_LAUNCH:
                assert acc, "op %s records no accesses" % name
                assert all(n > 0 for _, n, _ in acc)
    assert "adam_gd" in names or {"adam_g", "adam_d"} <= names
    assert any(n.startswith("d_head") and n.endswith("+loss") for n in names)
    launches = sum(p.op_info(i)[2] == eng.ext.OP_LAUNCH for p in (eng.progA, eng.progB, eng.progW, eng.progC)
                   for i in range(p.size()))
    assert eng.kernel_count() == launches


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_adam_g_split_has_no_hazards(monkeypatch, split, wire):
    """Segmented DDP step with Adam over g_h1's slice right after its collective (and the rest of
    Adam(G) after the last one) -- and without the split: no unordered overlaps, any wire."""
    monkeypatch.setenv("DCGAN_DDP_SHARD", "0")  # the all-reduce segmented step
    monkeypatch.setenv("DCGAN_ADAM_G_SPLIT", split)
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=2, dry_run=True, graph=False,
                    allreduce_dtype=wire)
    names = [n for n, _, _ in eng._segments()]
    assert ("adam_G_a" in names) == (split == "1"), names
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_checker_finds_adam_g_a_before_its_collective(monkeypatch):
    """Adam over g_h1's slice issued without waiting for that slice's collective: the checker
    reports the race on the gradient slice."""
    monkeypatch.setenv("DCGAN_DDP_SHARD", "0")  # the all-reduce segmented step
    eng = _dry(world=2)
    names = [n for n, _, _ in eng._segments()]
    assert names.index("adam_G_a") == 5

    def racy(ex):
        cs, alt = ex.main(), ex.alt[0]
        eng._seg(ex, 0, cs)
        ex.wait(alt, cs)
        eng._seg(ex, 1, alt)
        eng._ar_launch(ex, "dtop", alt)
        eng._seg(ex, 2, cs)
        eng._ar_launch(ex, "gsplit_a", cs)
        eng._seg(ex, 3, alt)
        eng._seg(ex, 4, cs)
        eng._seg(ex, 5, cs)                  # no wait for gsplit_a's collective
        eng._ar_launch(ex, "drest", alt)
        eng._ar_launch(ex, "gsplit_b", cs)
        eng._ar_launch(ex, "gsplit_c", cs)
        ex.wait(cs, alt)
        eng._ar_join(ex, cs)
        eng._seg(ex, 6, cs)
        eng._seg(ex, 7, cs)

    eng._run_step = racy
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed Adam(g_h1) racing its all-reduce"


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_ddp_gw_alt_has_no_hazards(monkeypatch, wire):
    """The segmented DDP step with G's weight gradients (but g_h1's) on the idle alt1 stream as
    soon as their operands exist; any wire."""
    monkeypatch.setenv("DCGAN_DDP_SHARD", "0")  # the all-reduce segmented step
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=2, dry_run=True, graph=False,
                    allreduce_dtype=wire)
    assert eng._schedule() == "concurrent" and eng._ddp_gw_alt()
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))



def test_checker_finds_ddp_g_bucket_before_the_alt1_weight_gradients(monkeypatch):
    """G's slice above g_h1 put on the wire from cs instead of from alt1 (i.e. without waiting
    for the weight gradients running there): the checker reports the race."""
    monkeypatch.setenv("DCGAN_DDP_SHARD", "0")  # the all-reduce segmented step
    eng = _dry(world=2)
    orig = eng._ar_launch

    def launch(ex, which, src):
        orig(ex, which, ex.main() if which == "gsplit_b" else src)

    eng._ar_launch = launch
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed G's collective racing the alt1 weight gradients"


def test_checker_finds_an_early_g_bucket_one_graph():
    """One-graph DDP: issuing G's first bucket one weight-gradient piece too early (before the
    piece that finalises it) is a race between the collective and that wgrad."""
    eng = _dry(world=2, schedule="ddp")
    assert eng._schedule() == "ddp"
    hz, _ = SC.check_engine(eng)
    assert hz == []
    k, lo, hi = eng._g_cuts[0]
    assert k >= 1
    eng._g_cuts[0] = (k - 1, lo, hi)
    hz, _ = SC.check_engine(eng)
    assert any("allreduce" in h.a or "allreduce" in h.b for h in hz), hz


def test_ddp_g_buckets_tile_the_gradient():
    eng = _dry(world=2, schedule="ddp")
    cuts = eng._g_cuts
    assert len(cuts) == 3 and cuts[-1][1] == 0
    assert cuts[0][2] == eng.grad_g.flat.numel()
    for (_, lo, _), (_, _, hi) in zip(cuts, cuts[1:]):
        assert lo == hi


@pytest.mark.parametrize("bad", ["fused", "concurent", "graph"])
def test_bad_ddp_schedule_env_is_rejected(monkeypatch, bad):
    """DCGAN_DDP_SCHEDULE must name a schedule that issues the all-reduces: 'fused' would train
    the ranks independently, a typo would run the serial code over the concurrent segments."""
    monkeypatch.setenv("DCGAN_DDP_SCHEDULE", bad)
    with pytest.raises(ValueError, match="DCGAN_DDP_SCHEDULE"):
        _dry(world=2)


@pytest.mark.parametrize("good", ["ddp", "concurrent", "serial"])
def test_ddp_schedule_env_selects_the_schedule(monkeypatch, good):
    monkeypatch.setenv("DCGAN_DDP_SCHEDULE", good)
    eng = _dry(world=2)
    assert eng._schedule() == good
    hz, _ = SC.check_engine(eng)
    assert hz == []








@pytest.mark.parametrize("place", ["sasa", "ssac", "dsac", "sdcc", "aaaa", "cccc", "dddd"])
def test_fused_g_wgrad_placements_have_no_hazards(monkeypatch, place):
    """DCGAN_GW_PLACE: G weight-gradient segments spread over the D chain's stream, cs and both
    idle streams (two weight gradients may run at once: no shared workspace between them)."""
    monkeypatch.setenv("DCGAN_GW_PLACE", place)
    eng = _dry()
    assert eng._gw_place() == place
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))






def test_fused_g_wgrad_place_rejects_bad_values(monkeypatch):
    for bad in ("ss", "sxsc"):
        monkeypatch.setenv("DCGAN_GW_PLACE", bad)
        with pytest.raises(ValueError):
            _dry()._gw_place()




def test_checker_finds_an_early_g_bucket(monkeypatch):
    """Segmented DDP: issuing the all-reduce of g_h1's slice before the G chain segment that
    computes its weight gradient is a race the checker reports."""
    monkeypatch.setenv("DCGAN_DDP_SHARD", "0")  # the all-reduce segmented step
    eng = _dry(world=2)

    def early(ex):
        cs, alt = ex.main(), ex.alt[0]
        eng._seg(ex, 0, cs)
        ex.wait(alt, cs)
        eng._seg(ex, 1, alt)
        eng._ar_launch(ex, "gsplit_a", cs)   # too early: G_chain has not run
        for i, st in ((2, cs), (3, alt), (4, cs)):
            eng._seg(ex, i, st)
        ex.wait(cs, alt)
        eng._ar_join(ex, cs)
        for i in range(5, len(eng._segments())):
            eng._seg(ex, i, cs)

    eng._run_step = early
    hz, _ = SC.check_engine(eng)
    assert any("allreduce" in h.a or "allreduce" in h.b for h in hz), hz


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("schedule", [None, "serial", "ddp"])
def test_bf16_wire_schedules_have_no_hazards(dtype, schedule):
    """bf16 wire: the segmented step's in-graph casts + in-place reduced bf16 images read by
    Adam (bf16 engine), and the reducer's copying path (other schedules / the fp16 engine)."""
    sched, hz, n = SC.check(DCGANConfig(), 4, dtype, 2, schedule, False, allreduce_dtype="bf16")
    assert n > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_bf16_wire_direct_path_is_used(monkeypatch):
    monkeypatch.setenv("DCGAN_DDP_SHARD", "0")  # the all-reduce segmented step
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=2, dry_run=True, graph=False, allreduce_dtype="bf16")
    assert eng._schedule() == "concurrent" and eng._wire_direct()
    assert {"dtop", "drest", "g_a", "g_b", "g_c"} <= set(eng._wire_ops)
    eng._ensure_comm()
    assert eng._ar_dtop.prefilled and eng._ar_gsplit_a.prefilled and eng._ar_gsplit_c.prefilled
    # the collective no longer touches the fp32 gradient, only its bf16 image
    assert all(p != eng.grad_d.flat.data_ptr() for p, _, _ in eng._ar_drest.accesses())
    names = [eng.progC.op_info(i)[0] for i in range(eng.progC.size())]
    assert "adam_d" in names and {"adam_g_a", "adam_g_b", "adam_g_c"} <= set(names)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_update_is_hazard_free(world, monkeypatch):
    """Segmented DDP step, bf16, eager, DCGAN_DDP_SHARD=1: the conv kernels go reduce-scatter ->
    Adam on 1/W -> all-gather of the bf16 mirror (4 slices), the fp32-read tensors through two
    all-reduces. (Opt-in: the per-slice all-reduce step measured faster under the stand-in,
    profiles/r6/ab_ddp_shard_standin_r6.txt.)"""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    monkeypatch.setenv("DCGAN_DDP_SHARD", "1")
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=world, dry_run=True, graph=False)
    assert eng._sharded() and sorted(eng._shards) == ["dw_rest", "dw_top", "g_a", "g_b"]
    assert [n for n, _, _, _ in eng._small] == ["d_small", "g_c"]
    for name, (sr, m, a, b) in eng._shards.items():
        assert sr.n * world == b - a and sr.lo == 0
    hz, n = SC.check_engine(eng)
    assert n > 100 and hz == [], "\n".join(map(str, hz[:10]))


def test_checker_finds_the_top_kernel_gather_before_its_last_reader(monkeypatch):
    """The top D kernel's Adam + all-gather must follow the D chain's top-layer data gradient
    (it reads the old bf16 mirror): issued right after its reduce-scatter, the checker reports it."""
    monkeypatch.setenv("DCGAN_DDP_SHARD", "1")
    eng = _dry(world=2)
    assert eng._sharded()

    def early(ex):
        cs, alt = ex.main(), ex.alt[0]
        eng._seg(ex, 0, cs)
        ex.wait(alt, cs)
        eng._seg(ex, 1, alt)
        eng._sh_rs(ex, "dw_top", alt)
        eng._sh_update(ex, "dw_top")          # too early: the top-layer dgrad has not run
        eng._g_chain_gw_alt(ex, cs, sharded=True)
        eng._sh_rs(ex, "g_a", cs)
        eng._sh_update(ex, "g_b")
        ex.run(eng.progB, ex.alt, eng._b_split, -1)
        eng._sh_rs(ex, "dw_rest", alt)
        eng._sh_update(ex, "dw_rest")
        eng._ar_launch(ex, "d_small", alt)
        eng._g_tail_gw_alt(ex, cs)
        eng._ar_launch(ex, "g_c", cs)
        eng._sh_update(ex, "g_a")
        eng._ar_join(ex, cs)
        ex.wait(cs, alt)
        eng._seg(ex, 5, cs)

    eng._run_step = early
    hz, _ = SC.check_engine(eng)
    assert any("all_gather" in h.a or "all_gather" in h.b for h in hz), "\n".join(map(str, hz[:10]))
