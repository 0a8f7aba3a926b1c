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
        eng._build() if eng._wgrad_adam else eng._build_updates()
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
    assert ("adam_gd" in names or "adam_rest" in names or {"adam_g", "adam_d"} <= names
            or {"adam_gd_a", "adam_g_b"} <= names)
    assert any(n.startswith("d_head") and n.endswith("+loss") for n in names)
    launches = sum(p.op_info(i)[2] == eng.ext.OP_LAUNCH for p in (eng.progA, eng.progB, eng.progW, eng.progC)
                   for i in range(p.size()))
    assert eng.kernel_count() == launches


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_adam_g_split_has_no_hazards(monkeypatch, split, wire):
    """Segmented DDP step with Adam over g_h1's slice right after its collective (and the rest of
    Adam(G) after the last one) -- and without the split: no unordered overlaps, any wire."""
    monkeypatch.setenv("DCGAN_ADAM_G_SPLIT", split)
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=2, dry_run=True, graph=False,
                    allreduce_dtype=wire)
    names = [n for n, _, _ in eng._segments()]
    assert ("adam_G_a" in names) == (split == "1"), names
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_checker_finds_adam_g_a_before_its_collective():
    """Adam over g_h1's slice issued without waiting for that slice's collective: the checker
    reports the race on the gradient slice."""
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


@pytest.mark.parametrize("mode", ["1", "2", "3"])
@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_ddp_gw_alt_has_no_hazards(monkeypatch, mode, wire):
    """DCGAN_DDP_GW_ALT=1/2: the segmented DDP step with G's weight gradients (2: g_h1's too) on
    the idle alt1 stream as soon as their operands exist; any wire."""
    monkeypatch.setenv("DCGAN_DDP_GW_ALT", mode)
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=2, dry_run=True, graph=False,
                    allreduce_dtype=wire)
    assert eng._schedule() == "concurrent" and eng._ddp_gw_alt() == int(mode)
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


@pytest.mark.parametrize("mode", ["1", "2", "3"])
def test_gw_alt_timed_single_process_has_no_hazards(monkeypatch, mode):
    """W=1 with phase timers (the segmented step without collectives, so no comm-stream joins):
    every DCGAN_DDP_GW_ALT mode still joins its streams into cs."""
    monkeypatch.setenv("DCGAN_DDP_GW_ALT", mode)
    eng = _dry(timing=True)
    assert eng._schedule() == "concurrent" and not eng.ddp and eng._ddp_gw_alt() == int(mode)
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_ddp_dmid_has_no_hazards(monkeypatch, wire):
    """DCGAN_DDP_DMID=1: D's gradient in three collectives (top layer + head; the next layer down
    as soon as its weight gradient lands; the rest at the D chain's end)."""
    monkeypatch.setenv("DCGAN_DDP_DMID", "1")
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    eng = HipEngine(DCGANConfig(), 4, torch.device("cpu"), world=2, dry_run=True, graph=False,
                    allreduce_dtype=wire)
    eng._ensure_comm()
    assert eng._ddp_dmid() and eng._b_split < eng._b_split2
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_checker_finds_ddp_dmid_before_its_weight_gradient(monkeypatch):
    """The D-mid collective issued one op too early (before the weight gradient that finalises
    its slice) is a race the checker reports."""
    monkeypatch.setenv("DCGAN_DDP_DMID", "1")
    eng = _dry(world=2)
    eng._ensure_comm()
    assert eng._ddp_dmid()
    eng._b_split2 -= 1
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed D's middle collective racing its weight gradient"


def test_checker_finds_ddp_g_bucket_before_the_alt1_weight_gradients(monkeypatch):
    """DCGAN_DDP_GW_ALT=1 with G's slice above g_h1 put on the wire from cs instead of from alt1
    (i.e. without waiting for the weight gradients running there): the checker reports the race."""
    monkeypatch.setenv("DCGAN_DDP_GW_ALT", "1")
    eng = _dry(world=2)
    orig = eng._ar_launch

    def launch(ex, which, src):
        orig(ex, which, ex.main() if which == "gsplit_b" else src)

    eng._ar_launch = launch
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed G's collective racing the alt1 weight gradients"


def test_checker_finds_an_early_g_bucket():
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


@pytest.mark.parametrize("wa", ["0", "1"])
def test_wgrad_adam_schedule_has_no_hazards(monkeypatch, wa):
    monkeypatch.setenv("DCGAN_WGRAD_ADAM", wa)
    eng = _dry()
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_early_adam_d_has_no_hazards(monkeypatch):
    """DCGAN_ADAM_D_EARLY=1: Adam(D) on the D chain's stream (after the g_loss chain has left D)
    beside the G chain's tail -- no unordered overlap with the G chain's reads of D's weights."""
    monkeypatch.setenv("DCGAN_ADAM_D_EARLY", "1")
    eng = _dry()
    assert eng._adam_early and eng._schedule() == "fused"
    names = [eng.progC.op_info(i)[0] for i in range(eng.progC.size())]
    assert names[:eng._c_split] == ["adam_d"]
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_checker_finds_adam_d_before_the_g_chain_left_d(monkeypatch):
    """The same Adam(D) issued on the D chain's stream WITHOUT waiting for the g_loss chain to leave
    D races the G chain's D data gradients (they read D's weights)."""
    monkeypatch.setenv("DCGAN_ADAM_D_EARLY", "1")
    eng = _dry()

    def racy(ex):
        cs, alt = ex.main(), ex.alt[0]
        ex.run(eng.progA, [cs, ex.side], 0, eng._a_fwd)
        ex.wait(alt, cs)
        ex.run(eng.progB, ex.alt)
        ex.run(eng.progC, ex.alt, 0, eng._c_split)    # Adam(D): no wait for the g_loss chain
        ex.run(eng.progA, [cs, ex.side], eng._a_fwd, -1)
        ex.run(eng.progW, [cs, ex.side])
        ex.wait(cs, alt)
        ex.run(eng.progC, [cs, ex.side], eng._c_split, -1)

    eng._run_step = racy
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed Adam(D) racing the g_loss chain's reads of D"


@pytest.mark.parametrize("fold", ["0", "64", "256"])
def test_bn_fold_schedule_has_no_hazards(monkeypatch, fold):
    """BN finalize folded into the apply launches (DCGAN_BN_FOLD): same hazard-free step, one
    launch fewer per folded layer."""
    monkeypatch.setenv("DCGAN_BN_FOLD", fold)
    eng = _dry()
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))
    names = [eng.progA.op_info(i)[0] for i in range(eng.progA.size())]
    names += [eng.progB.op_info(i)[0] for i in range(eng.progB.size())]
    n_fold = sum(1 for n in names if n.endswith("fin_apply"))
    assert (n_fold == 0) == (fold == "0"), n_fold


@pytest.mark.parametrize("n", ["0", "1", "2", "4"])
def test_fused_g_wgrad_tail_on_main_has_no_hazards(monkeypatch, n):
    """DCGAN_GW_TAIL_ON_MAIN=n: the last n G weight gradients of the fused step on the G chain's
    stream after that chain -- still free of unordered overlaps."""
    monkeypatch.setenv("DCGAN_GW_TAIL_ON_MAIN", n)
    eng = _dry()
    assert eng._schedule() == "fused" and eng._gw_tail_on_main() == int(n)
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


@pytest.mark.parametrize("where", ["side", "alt1"])
@pytest.mark.parametrize("n", ["0", "2"])
def test_fused_g_wgrad_stream_has_no_hazards(monkeypatch, where, n):
    """DCGAN_GW_STREAM=side/alt1: the G weight gradients on an otherwise idle stream beside both
    chains (each after its operand's mark), joined into cs before Adam."""
    monkeypatch.setenv("DCGAN_GW_STREAM", where)
    monkeypatch.setenv("DCGAN_GW_TAIL_ON_MAIN", n)
    eng = _dry()
    assert eng._gw_place() == where[0] * (4 - int(n)) + "c" * int(n)
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


@pytest.mark.parametrize("place", ["sasa", "ssac", "dsac", "sdcc", "aaaa"])
def test_fused_g_wgrad_placements_have_no_hazards(monkeypatch, place):
    """DCGAN_GW_PLACE: G weight-gradient segments spread over the D chain's stream, cs and both
    idle streams (two weight gradients may run at once: no shared workspace between them)."""
    monkeypatch.setenv("DCGAN_GW_PLACE", place)
    eng = _dry()
    assert eng._gw_place() == place
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_adam_split_alt_is_hazard_free(monkeypatch):
    """DCGAN_ADAM_SPLIT_ALT=1, fused bf16 step: Adam over D and G from g_h2 on runs on the weight
    gradients' stream beside the G chain's tail (progC[:_c_split]); the rest + the beta powers
    after the join."""
    monkeypatch.setenv("DCGAN_ADAM_SPLIT_ALT", "1")
    eng = _dry()
    assert eng._adam_alt and eng._c_split == 1
    assert [eng.progC.op_info(i)[0] for i in range(eng.progC.size())] == ["adam_gd_a", "adam_g_b"]
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_checker_finds_adam_part_before_the_d_chain_ended(monkeypatch):
    """The same first Adam part issued WITHOUT waiting for the D chain races D's weight
    gradients (and the D chain's reads of D's weights)."""
    monkeypatch.setenv("DCGAN_ADAM_SPLIT_ALT", "1")
    eng = _dry()

    def racy(ex):
        cs, a1 = ex.main(), ex.alt[1]
        ex.run(eng.progA, [cs, ex.side], 0, eng._a_fwd)
        ex.wait(ex.alt[0], cs)
        ex.run(eng.progB, ex.alt)
        pos, w = eng._a_fwd, 0
        for a_end, w_end in eng._g_w:
            ex.run(eng.progA, [cs, ex.side], pos, a_end)
            ex.wait(a1, cs)
            ex.run(eng.progW, [a1], w, w_end)
            pos, w = a_end, w_end
        ex.run(eng.progA, [cs, ex.side], pos, -1)
        ex.run(eng.progC, [a1], 0, eng._c_split)   # no wait for the D chain
        ex.wait(cs, a1)
        ex.wait(cs, ex.alt[0])
        ex.run(eng.progC, [cs, ex.side], eng._c_split, -1)

    eng._run_step = racy
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed Adam(D) racing the D chain"


def test_checker_finds_adam_part_over_g_h1(monkeypatch):
    """A first Adam part that also covers g_h1's weights races the G chain's g_h1 data gradient
    (it reads g_h1's 16-bit mirror after the last weight-gradient mark)."""
    monkeypatch.setenv("DCGAN_ADAM_SPLIT_ALT", "1")
    eng = _dry()
    lo = eng.model.g.offsets[eng.gl[0].name + "/w"][0]
    G, og = eng.model.g, eng.opt_g
    eng.progC = eng._prog()
    eng.progC.adam2_part("bad", G.flat.data_ptr() + 4 * lo, eng.wbf_g.flat.data_ptr() + 2 * lo,
                         eng.grad_g.flat.data_ptr() + 4 * lo, og.m.flat.data_ptr() + 4 * lo,
                         og.v.flat.data_ptr() + 4 * lo, og.powers.data_ptr(), G.flat.numel() - lo, 1e-3, 0.5,
                         0.999, 1e-8, 0, 0, 0, 0, 0, 0, 0, 1e-3, 0.5, 0.999, 1e-8, 1.0, 0)
    eng._c_split = 1
    hz, _ = SC.check_engine(eng)
    assert hz, "the checker missed Adam over g_h1 racing the g_h1 data gradient"


def test_d_wgrad_side_has_no_hazards(monkeypatch):
    """DCGAN_D_WGRAD_SIDE=1 (study): D's weight gradients on progB's slot-1 stream (the side
    stream in the fused step), each after its dx, joined back at the D chain's end."""
    monkeypatch.setenv("DCGAN_D_WGRAD_SIDE", "1")
    eng = _dry()
    assert eng._dws
    slots = {eng.progB.op_info(i)[1] for i in range(eng.progB.size())}
    assert slots == {0, 1}
    hz, _ = SC.check_engine(eng)
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_fused_g_wgrad_place_rejects_bad_values(monkeypatch):
    for bad in ("ss", "sxsc"):
        monkeypatch.setenv("DCGAN_GW_PLACE", bad)
        with pytest.raises(ValueError):
            _dry()._gw_place()


def test_fused_g_wgrad_tail_on_main_rejects_bad_values(monkeypatch):
    monkeypatch.setenv("DCGAN_GW_TAIL_ON_MAIN", "two")
    with pytest.raises(ValueError):
        _dry()._gw_tail_on_main()


@pytest.mark.parametrize("tail", ["0", "2", "4"])
def test_concurrent_ddp_gw_placements_have_no_hazards(monkeypatch, tail):
    """The segmented DDP step for every trailing-G-wgrad placement (DCGAN_GW_TAIL_ON_MAIN)."""
    monkeypatch.setenv("DCGAN_GW_TAIL_ON_MAIN", tail)
    eng = _dry(world=2)
    assert eng._schedule() == "concurrent"
    hz, n_ops = SC.check_engine(eng)
    assert n_ops > 100
    assert hz == [], "\n".join(map(str, hz[:10]))


def test_checker_finds_an_early_g_bucket():
    """Segmented DDP: issuing the all-reduce of g_h1's slice before the G chain segment that
    computes its weight gradient is a race the checker reports."""
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


def test_bf16_wire_direct_path_is_used():
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


def test_wgrad_adam_ranges_tile_both_buffers(monkeypatch):
    """DCGAN_WGRAD_ADAM=1, single-process bf16: the six conv / deconv weights get their TF-Adam
    in the wgrad3 store pass; the update pass covers every other element of both flat buffers
    exactly once (Adam) and re-writes the mirrors of the six (cast)."""
    monkeypatch.setenv("DCGAN_WGRAD_ADAM", "1")
    eng = _dry()
    assert eng._wgrad_adam and len(eng._adam_fused) == 2 * (len(eng.gl) - 1)
    names = [eng.progC.op_info(i)[0] for i in range(eng.progC.size())]
    assert names == ["adam_rest"]
    for s_, off, n in eng._adam_fused:
        ps = eng.model.g if s_ == 0 else eng.model.d
        assert any(o == off for o, _ in ps.offsets.values())
    d2 = _dry(timing=True)  # the timed (segmented) step re-records without it
    assert not d2._wgrad_adam and not d2._adam_fused
    names = [d2.progC.op_info(i)[0] for i in range(d2.progC.size())]
    assert "adam_rest" not in names


def test_wgrad_adam_is_off_by_default():
    eng = _dry()
    assert not eng._wgrad_adam
    names = [eng.progC.op_info(i)[0] for i in range(eng.progC.size())]
    assert names == (["adam_gd_a", "adam_g_b"] if eng._adam_alt else ["adam_gd"])
