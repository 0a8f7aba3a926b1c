"""Whole-step parity of the fused HIP engine (MI355X only).

Two kinds of checks:

* ``test_engine_stagewise``: every backward stage of the engine (head dgrad, BN+act backward,
  conv/deconv dgrad, wgrad, G projection grads) is recomputed in fp64 from the engine's OWN
  stage inputs and compared tightly. This isolates kernel correctness from mixed-precision
  drift.
* ``test_engine_step_matches_reference``: the whole step vs the fp32 autograd reference from
  the same init / z / real batch. Tolerances are loose on purpose: LeakyReLU/ReLU derivatives
  are discontinuous, so bf16-sized (0.3 %) differences in forward pre-activations flip the
  derivative mask of near-zero elements and move BN-backward outputs by ~2 % per layer (measured:
  0.3 % input perturbation -> 2 % dx change); this compounds through the 8-layer D->G chain.
"""
import pytest
import torch

from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig, same_pads
from distributed_tensorflow_for_dcgan_amd.models.dcgan import DCGAN
from distributed_tensorflow_for_dcgan_amd.engine.reference_step import ReferenceStep
from distributed_tensorflow_for_dcgan_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().flatten().cpu(), b.double().flatten().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def d64(t):
    return t.detach().double()


def w64(t, edt=torch.bfloat16):
    """weights as the kernels see them (the bf16 / fp16 mirror)"""
    return t.detach().to(edt).double()


def bn_act_bwd64(x, dy, gamma, beta, act, groups=1):
    x = d64(x).clone().requires_grad_(True)
    C = x.shape[-1]
    xg = x.reshape(groups, -1, C)
    m = xg.mean(1, keepdim=True)
    v = (xg - m).pow(2).mean(1, keepdim=True)
    u = ((xg - m) / torch.sqrt(v + 1e-5) * d64(gamma) + d64(beta)).reshape(x.shape)
    a = torch.relu(u) if act == "relu" else torch.maximum(u, 0.2 * u)
    gx, = torch.autograd.grad(a, x, d64(dy))
    ug = u.detach().reshape(-1, C)
    dyg = d64(dy).reshape(-1, C) * (torch.where(ug > 0, 1.0, 0.0 if act == "relu" else 0.2))
    xhat = ((xg - m) / torch.sqrt(v + 1e-5)).detach().reshape(-1, C)
    return gx, (dyg * xhat).sum(0), dyg.sum(0)


def conv_grads64(x, w, dy, kind, out_hw=None, edt=torch.bfloat16):
    """(dx, dw) of a TF-SAME conv (kind 'conv', HWIO w) or conv_transpose ('deconv')."""
    xv = d64(x).clone().requires_grad_(True)
    wv = w64(w, edt).clone().requires_grad_(True)
    if kind == "conv":
        y = R.conv2d_same(xv, wv)
    else:
        y = R.conv2d_transpose_same(xv, wv, out_hw)
    return torch.autograd.grad(y, [xv, wv], d64(dy))


def _lrelu_d(a):
    a = d64(a)
    return torch.where(a > 0, torch.ones_like(a), torch.full_like(a, 0.2))


@pytest.mark.parametrize("size,c_dim,B,dtype", [(64, 3, 16, "bf16"), (28, 1, 8, "bf16"), (128, 3, 4, "bf16"),
                                                (256, 3, 4, "bf16"), (64, 3, 16, "fp16"), (256, 3, 4, "fp16"),
                                                (64, 3, 8, "fp32"), (28, 1, 8, "fp32")])
def test_engine_stagewise(size, c_dim, B, dtype, monkeypatch):
    """fp16 runs with the dynamic loss scale in the gradient seeds: every stage is compared
    against a recomputation from the engine's own (scaled) inputs, so the scale cancels.
    Programs A / B / W hold no optimiser op: the G stages are recomputed from the pre-update G
    weights. fp32 (the reference precision) is held
    to 1e-4 per stage."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    from distributed_tensorflow_for_dcgan_amd.ops import hip as H
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig(output_size=size, c_dim=c_dim)
    eng = HipEngine(cfg, B, dev, graph=False, seed=3, dtype=dtype)
    edt = eng.edt
    real = (torch.rand(B, size, size, c_dim, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(dev)
    eng.set_batch(real)
    st = [torch.cuda.current_stream(), torch.cuda.Stream()]  # main + side stream slots
    H.run(eng.progA, st)          # forward, g_loss chain through D(fake), G data gradients
    H.run(eng.progW, st)          # G weight gradients (G grads final)
    torch.cuda.synchronize()
    Pd, Pg, gD, gG = eng.model.d, eng.model.g, eng.grad_d, eng.grad_g
    rep = {}
    dl, gl = cfg.d_layers(), cfg.g_layers()
    lin = cfg.d_lin_name
    B2 = 2 * B
    for i in range(len(dl) - 1, -1, -1):
        L = dl[i]
        if L.bn:
            gx, _, _ = bn_act_bwd64(eng.d_x[L.name][B:], eng.gc_da[L.name], Pd[L.bn + "/gamma"],
                                    Pd[L.bn + "/beta"], "lrelu")
            rep["g %s bn dx" % L.name] = rel(eng.gc_dx[L.name], gx)
        src = eng.d_in[B:] if i == 0 else eng.d_a[dl[i - 1].name][B:]
        gx, _ = conv_grads64(src, Pd[L.name + "/w"], eng.gc_dx[L.name], "conv", edt=edt)
        if i == 0 and eng._img_dact():  # G's tanh backward fused into the image-gradient kernel
            fk = d64(eng.fake)
            rep["g %s dgrad+tanh bwd" % L.name] = rel(eng.img_g, gx * (1 - fk * fk))
        elif i == 0:
            rep["g %s dgrad" % L.name] = rel(eng.img_grad, gx)
        elif dl[i - 1].bn:
            rep["g %s dgrad" % L.name] = rel(eng.gc_da[dl[i - 1].name], gx)
        else:  # the act backward of a BN-less layer is fused into this GEMM: it stores dx
            rep["g %s dgrad+act" % L.name] = rel(eng.gc_dx[dl[i - 1].name], gx * _lrelu_d(eng.d_a[dl[i - 1].name][B:]))
    fake = d64(eng.fake)
    if eng._img_dact():
        img_g = d64(eng.img_g)  # checked above against the oracle; the bias gradient sums it
    else:
        img_g = d64(eng.img_grad) * (1 - fake * fake)
        rep["G tanh bwd"] = rel(eng.img_g, img_g)
    for j in range(len(gl) - 1, -1, -1):
        L = gl[j]
        src = eng.g_a[gl[j - 1].name] if j > 0 else eng.g_h0
        dy = eng.img_g if not L.bn else eng.g_dx[L.name]
        if L.bn:
            gx, dgam, dbet = bn_act_bwd64(eng.g_x[L.name], eng.g_da[L.name], Pg[L.bn + "/gamma"], Pg[L.bn + "/beta"],
                                          "relu")
            rep["G %s bn dx" % L.name] = rel(eng.g_dx[L.name], gx)
            rep["G %s dgamma" % L.bn] = rel(gG[L.bn + "/gamma"], dgam)
            rep["G %s dbeta" % L.bn] = rel(gG[L.bn + "/beta"], dbet)
        Bx = src.reshape(B, L.in_hw, L.in_hw, L.cin)
        gx, gw = conv_grads64(Bx, Pg[L.name + "/w"], dy, "deconv", (L.out_hw, L.out_hw), edt=edt)
        rep["G %s dW" % L.name] = rel(gG[L.name + "/w"], gw)
        dsrc = eng.g_da[gl[j - 1].name] if j > 0 else eng.g_da0
        rep["G %s dgrad" % L.name] = rel(dsrc.reshape(gx.shape), gx)
    rep["G out dbias"] = rel(gG[gl[-1].name + "/biases"], img_g.reshape(-1, cfg.c_dim).sum(0))
    gx, dgam, dbet = bn_act_bwd64(eng.g_h0_pre.reshape(B, cfg.g_base_hw, cfg.g_base_hw, cfg.g_base_ch),
                                  eng.g_da0.reshape(B, cfg.g_base_hw, cfg.g_base_hw, cfg.g_base_ch),
                                  Pg["g_bn0/gamma"], Pg["g_bn0/beta"], "relu")
    rep["G bn0 dx"] = rel(eng.g_dx0.reshape(gx.shape), gx)
    rep["G lin dW"] = rel(gG["g_h0_lin/Matrix"], d64(eng.z).t() @ d64(eng.g_dx0))
    rep["G lin db"] = rel(gG["g_h0_lin/bias"], d64(eng.g_dx0).sum(0))
    H.run(eng.progB, st)          # D backward of d_loss
    torch.cuda.synchronize()
    # head
    a_last = d64(eng.d_a[dl[-1].name]).reshape(B2, -1)
    rep["d head dW"] = rel(gD[lin + "/Matrix"].flatten(), a_last.t() @ d64(eng.dl_d))
    rep["d head da"] = rel(eng.d_da[dl[-1].name].reshape(B2, -1), d64(eng.dl_d)[:, None] * d64(Pd[lin + "/Matrix"]).t())
    for i in range(len(dl) - 1, -1, -1):
        L = dl[i]
        if L.bn:
            gx, dgam, dbet = bn_act_bwd64(eng.d_x[L.name], eng.d_da[L.name], Pd[L.bn + "/gamma"], Pd[L.bn + "/beta"],
                                          "lrelu", groups=2)
            rep["d %s bn dx" % L.name] = rel(eng.d_dx[L.name], gx)
            rep["d %s dgamma" % L.bn] = rel(gD[L.bn + "/gamma"], dgam)
            rep["d %s dbeta" % L.bn] = rel(gD[L.bn + "/beta"], dbet)
        src = eng.d_in if i == 0 else eng.d_a[dl[i - 1].name]
        gx, gw = conv_grads64(src, Pd[L.name + "/w"], eng.d_dx[L.name], "conv", edt=edt)
        rep["d %s dW" % L.name] = rel(gD[L.name + "/w"], gw)
        if i > 0:
            if dl[i - 1].bn:
                rep["d %s dgrad" % L.name] = rel(eng.d_da[dl[i - 1].name], gx)
            else:
                rep["d %s dgrad+act" % L.name] = rel(eng.d_dx[dl[i - 1].name], gx * _lrelu_d(eng.d_a[dl[i - 1].name]))
    rep["d h0 dbias"] = rel(gD[dl[0].name + "/biases"], d64(eng.d_dx[dl[0].name]).reshape(-1, dl[0].cout).sum(0))
    print("\nstagewise relative errors (%dx%dx%d, B=%d, %s):" % (size, size, c_dim, B, dtype))
    for k, v in rep.items():
        print("  %-28s %.5f" % (k, v))
    # BN-backward stages see derivative-mask flips of near-zero bf16 pre-activations -> 3 %
    if dtype == "fp32":
        bad = {k: v for k, v in rep.items() if v > 1e-4}
    else:
        bad = {k: v for k, v in rep.items() if v > (0.03 if ("bn dx" in k or "dbeta" in k) else 0.01)}
    assert not bad, bad


@pytest.mark.parametrize("size,c_dim,B", [(64, 3, 16), (28, 1, 8), (32, 3, 8), (128, 3, 8), (256, 3, 8)])
def test_engine_step_matches_reference(size, c_dim, B):
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig(output_size=size, c_dim=c_dim)
    eng = HipEngine(cfg, B, dev, graph=False, seed=3)
    real = (torch.rand(B, size, size, c_dim, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(dev)
    real = real.to(torch.bfloat16).float()
    eng.set_batch(real)
    ref_model = DCGAN(cfg, device=dev, seed=3)
    assert torch.equal(ref_model.g.flat, eng.model.g.flat)
    eng.train_step()
    torch.cuda.synchronize()
    out, gd, gg = ReferenceStep(ref_model).compute_grads(real, eng.z.clone())
    L = eng.last_losses()
    for k in ("d_loss_real", "d_loss_fake", "g_loss", "d_loss"):
        r = float(out[k].detach())
        assert abs(L[k] - r) <= 3e-2 * max(1.0, abs(r)), (k, L[k], r)
    gdref, ggref = ref_model.d.like(), ref_model.g.like()
    gdref.flat.copy_(gd)
    ggref.flat.copy_(gg)
    gl_last = cfg.g_layers()[-1].name
    errs = {}
    for name in ref_model.d.names():
        if name.endswith("/biases") and not name.startswith("d_h0_conv"):
            continue  # dead bias (followed by BN)
        errs[name] = rel(eng.grad_d[name], gdref[name])
    for name in ref_model.g.names():
        if name.endswith("/biases") and name.split("/")[0] != gl_last:
            continue
        errs[name] = rel(eng.grad_g[name], ggref[name])
    print("\nend-to-end relative grad errors vs fp32 reference (%dx%dx%d, B=%d):" % (size, size, c_dim, B))
    for k, v in errs.items():
        print("  %-28s %.4f" % (k, v))
    small_sums = {gl_last + "/biases"}  # 3-element sums over all pixels: heavy cancellation
    # the live D layer-0 bias is a sum of dx over every pixel (cancellation as well): at depth 6
    # (256x256) its bf16 end-to-end error sits near the weight errors' upper range
    tol = {k: (0.35 if k.endswith("/biases") else 0.25) for k in errs}
    bad = {k: v for k, v in errs.items() if v > tol[k] and k not in small_sums}
    assert not bad, bad
    # bf16 activations + ReLU/LeakyReLU mask flips compound with depth (each stage is checked
    # to <= 1-3 % against fp64 on the engine's own tensors in test_engine_stagewise)
    assert sum(errs.values()) / len(errs) < (0.15 if len(cfg.d_layers()) <= 4 else 0.2)
    for name, _ in cfg.g_bn_layers():
        assert rel(eng.model.g_bn.mean[name], ref_model.g_bn.mean[name]) < 5e-2, name
        assert rel(eng.model.g_bn.var[name], ref_model.g_bn.var[name]) < 5e-2, name
    for name, _ in cfg.d_bn_layers():
        assert rel(eng.model.d_bn.var[name], ref_model.d_bn.var[name]) < 5e-2, name
    assert eng.global_step == 1
    assert abs(float(eng.opt_d.powers[0]) - 0.25) < 1e-7


def test_engine_adam_applies_tf_update():
    """Parameters after one step == TF-Adam applied to the engine's own gradients."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    eng = HipEngine(cfg, 8, dev, graph=False, seed=4)
    eng.set_batch((torch.rand(8, 64, 64, 3) * 2 - 1).to(dev))
    g0, d0 = eng.model.g.flat.clone(), eng.model.d.flat.clone()
    eng.train_step()
    torch.cuda.synchronize()
    for p0, p1, g in ((g0, eng.model.g.flat, eng.grad_g.flat), (d0, eng.model.d.flat, eng.grad_d.flat)):
        m = 0.5 * g  # (1 - beta1) * g with zero init
        v = 0.001 * g * g
        lr_t = 2e-4 * (1 - 0.999) ** 0.5 / (1 - 0.5)
        exp = p0 - lr_t * m / (v.sqrt() + 1e-8)
        assert torch.allclose(p1, exp, rtol=1e-5, atol=1e-7)


def test_engine_graph_replay_matches_eager():
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    B = 16
    real = (torch.rand(B, 64, 64, 3, generator=torch.Generator().manual_seed(1)) * 2 - 1).to(dev)
    e1 = HipEngine(cfg, B, dev, graph=False, seed=1)
    e2 = HipEngine(cfg, B, dev, graph=True, seed=1)
    e1.set_batch(real)
    e2.set_batch(real)
    for _ in range(4):
        e1.train_step()
        e2.train_step()
    torch.cuda.synchronize()
    assert e2.graph_enabled
    assert torch.equal(e1.model.g.flat, e2.model.g.flat)
    assert torch.equal(e1.model.d.flat, e2.model.d.flat)
    assert e1.last_losses() == e2.last_losses()
    assert e2.global_step == 4


def test_engine_sampler_and_eval():
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    B = 8
    eng = HipEngine(cfg, B, dev, graph=False, seed=2)
    real = (torch.rand(B, 64, 64, 3) * 2 - 1).to(dev)
    eng.set_batch(real)
    eng.train_step()
    z = (torch.rand(B, 100) * 2 - 1).to(dev)
    s = eng.sampler(z)
    ref = DCGAN(cfg, device=dev, seed=2)
    ref.g.flat.copy_(eng.model.g.flat)
    ref.g_bn.flat.copy_(eng.model.g_bn.flat)
    s_ref = ref.sampler(z)
    assert s.shape == (B, 64, 64, 3)
    assert rel(s, s_ref) < 5e-2
    before = eng.model.d_bn.flat.clone()
    ev = eng.eval_losses(real, z)
    assert torch.equal(before, eng.model.d_bn.flat)  # no EMA mutation
    assert ev["d_loss"] == ev["d_loss"]


def test_engine_fp16_loss_scaling():
    """fp16 engine: a good step keeps the scale and counts it; an overflowing step (scale forced
    to 1e38 -> inf gradients) is skipped -- weights, Adam slots, beta powers untouched -- and
    halves the scale; the step after trains again. Graph replay included."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    eng = HipEngine(cfg, 16, dev, seed=1, dtype="fp16")
    real = (torch.rand(16, 64, 64, 3, generator=torch.Generator().manual_seed(2)) * 2 - 1).to(dev)
    eng.set_batch(real)
    eng.train_step()
    eng.train_step()  # second step replays the captured graphs
    torch.cuda.synchronize()
    ls = eng.loss_scale.tolist()
    assert ls[0] == HipEngine.INIT_LOSS_SCALE and ls[1] == 0.0 and ls[2] == 2.0, ls
    assert all(torch.isfinite(torch.tensor(list(eng.last_losses().values()))))
    w0, m0 = eng.model.g.flat.clone(), eng.opt_g.m.flat.clone()
    p0 = eng.opt_d.powers.clone()
    eng.loss_scale[0] = 1e38
    eng.train_step()
    torch.cuda.synchronize()
    assert torch.equal(eng.model.g.flat, w0) and torch.equal(eng.opt_g.m.flat, m0)
    assert torch.equal(eng.opt_d.powers, p0)
    ls = eng.loss_scale.tolist()
    assert ls[0] == float(torch.tensor(1e38) * 0.5) and ls[1] == 0.0 and ls[2] == 0.0, ls
    eng.loss_scale[0] = 1024.0
    eng.train_step()
    torch.cuda.synchronize()
    assert not torch.equal(eng.model.g.flat, w0)
    assert eng.global_step == 4


def test_engine_fp16_step_matches_reference():
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    B = 16
    eng = HipEngine(cfg, B, dev, graph=False, seed=3, dtype="fp16")
    real = (torch.rand(B, 64, 64, 3, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(dev)
    real = real.to(torch.float16).float()
    eng.set_batch(real)
    ref_model = DCGAN(cfg, device=dev, seed=3)
    eng.train_step()
    torch.cuda.synchronize()
    out, gd, gg = ReferenceStep(ref_model).compute_grads(real, eng.z.clone())
    L = eng.last_losses()
    for k in ("d_loss_real", "d_loss_fake", "g_loss", "d_loss"):
        r = float(out[k].detach())
        assert abs(L[k] - r) <= 2e-2 * max(1.0, abs(r)), (k, L[k], r)
    scale = HipEngine.INIT_LOSS_SCALE  # raw engine grads carry the loss scale
    e_d = rel(eng.grad_d.flat / scale, gd)
    e_g = rel(eng.grad_g.flat / scale, gg)
    print("fp16 whole-step relative grad error: D %.4f G %.4f" % (e_d, e_g))
    assert e_d < 0.1 and e_g < 0.15


@pytest.mark.parametrize("size,c_dim,B", [(64, 3, 16), (28, 1, 8)])
def test_engine_fp32_step_matches_reference_tightly(size, c_dim, B):
    """The reference precision end to end on the HIP kernels (fp32 activations, fp32-input MFMA,
    igemm_f32.hip): one whole step (G fwd, D on real | fake, 3 losses, both backwards) against
    the fp32 autograd reference from the same init / z / batch -- every live gradient tensor
    within 1e-3 relative (dead biases, analytically zero, excluded), losses within 1e-5. The
    reference runs on the CPU: PyTorch's fp32 GPU convolutions (MIOpen) are not deterministic
    -- two reference runs differed by 6e-4 in G's gradients (benchmarks/det_check.py), while
    the HIP engine is bitwise reproducible."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig(output_size=size, c_dim=c_dim)
    eng = HipEngine(cfg, B, dev, graph=False, seed=3, dtype="fp32")
    assert eng.name == "hip" and eng.dtype_name == "fp32"
    real = (torch.rand(B, size, size, c_dim, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(dev)
    eng.set_batch(real)
    cpu = torch.device("cpu")
    ref_model = DCGAN(cfg, device=cpu, seed=3)
    eng.train_step()
    torch.cuda.synchronize()
    out, gd, gg = ReferenceStep(ref_model).compute_grads(real.cpu(), eng.z.cpu())
    L = eng.last_losses()
    for k in ("d_loss_real", "d_loss_fake", "g_loss", "d_loss"):
        r = float(out[k].detach())
        assert abs(L[k] - r) <= 1e-5 * max(1.0, abs(r)), (k, L[k], r)
    gdref, ggref = ref_model.d.like(), ref_model.g.like()
    gdref.flat.copy_(gd)
    ggref.flat.copy_(gg)
    gl_last = cfg.g_layers()[-1].name
    errs = {}
    for name in ref_model.d.names():
        if name.endswith("/biases") and not name.startswith("d_h0_conv"):
            continue  # dead bias (followed by BN)
        errs[name] = rel(eng.grad_d[name], gdref[name])
    for name in ref_model.g.names():
        if (name.endswith("/biases") and name.split("/")[0] != gl_last) or name == "g_h0_lin/bias":
            continue
        errs[name] = rel(eng.grad_g[name], ggref[name])
    print("\nfp32 end-to-end relative grad errors (%dx%dx%d, B=%d): max %.2e" % (size, size, c_dim, B,
                                                                               max(errs.values())))
    bad = {k: v for k, v in errs.items() if v > 1e-3}
    assert not bad, bad
    for name, _ in cfg.g_bn_layers():
        assert rel(eng.model.g_bn.mean[name], ref_model.g_bn.mean[name]) < 1e-5, name
        assert rel(eng.model.g_bn.var[name], ref_model.g_bn.var[name]) < 1e-5, name


def test_engine_fp32_graph_training_runs():
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    eng = HipEngine(DCGANConfig(), 16, dev, seed=1, dtype="fp32")
    eng.set_batch((torch.rand(16, 64, 64, 3, generator=torch.Generator().manual_seed(2)) * 2 - 1).to(dev))
    for _ in range(3):
        eng.train_step()
    torch.cuda.synchronize()
    assert eng.graph_enabled and eng.global_step == 3
    assert all(v == v for v in eng.last_losses().values())


def test_engine_sampler_zero_debias():
    """--bn_zero_debias on the HIP engine: the sampler divides G's moving averages by
    1 - decay^t (t = EMA updates so far), like the reference engine's BNState.averages."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    B = 8
    eng = HipEngine(cfg, B, dev, graph=False, seed=2, zero_debias=True)
    eng.set_batch((torch.rand(B, 64, 64, 3) * 2 - 1).to(dev))
    for _ in range(2):
        eng.train_step()
    z = (torch.rand(B, 100) * 2 - 1).to(dev)
    s = eng.sampler(z)
    ref = DCGAN(cfg, device=dev, seed=2, zero_debias=True)
    ref.g.flat.copy_(eng.model.g.flat)
    ref.g_bn.flat.copy_(eng.model.g_bn.flat)
    ref.g_bn.steps.copy_(eng.model.g_bn.steps)
    assert float(ref.g_bn.steps[0]) == 2
    s_ref = ref.sampler(z)
    ref_nodebias = DCGAN(cfg, device=dev, seed=2, zero_debias=False)
    ref_nodebias.g.flat.copy_(eng.model.g.flat)
    ref_nodebias.g_bn.flat.copy_(eng.model.g_bn.flat)
    assert rel(s, s_ref) < 5e-2
    assert rel(s, s_ref) < rel(s, ref_nodebias.sampler(z))




@pytest.mark.gpu
def test_g_wgrad_placements_are_bit_identical(monkeypatch):
    """The default G weight-gradient placement (idle alt1 stream, "aaaa") == round 4's (behind the
    D chain, last two on cs: "ddcc") == two idle streams ("sasa") == all on cs ("cccc"), bit for
    bit, 3 steps."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    B = 32
    real = (torch.rand(B, 64, 64, 3, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(dev)
    engs = []
    for place in (None, "ddcc", "sasa", "cccc"):
        if place is None:
            monkeypatch.delenv("DCGAN_GW_PLACE", raising=False)
        else:
            monkeypatch.setenv("DCGAN_GW_PLACE", place)
        e = HipEngine(DCGANConfig(), B, dev, graph=False, seed=5)
        e.set_batch(real)
        for _ in range(3):
            e.train_step()
        torch.cuda.synchronize()
        engs.append(e)
    monkeypatch.delenv("DCGAN_GW_PLACE", raising=False)
    assert engs[0]._gw_place() == "aaaa"
    assert all(e.global_step == 3 for e in engs)
    for e in engs[1:]:
        for a, b in ((engs[0].model.g.flat, e.model.g.flat), (engs[0].model.d.flat, e.model.d.flat),
                     (engs[0].opt_g.v.flat, e.opt_g.v.flat)):
            assert torch.equal(a, b), (a.float() - b.float()).abs().max()
        assert torch.equal(engs[0].wbf_g.flat, e.wbf_g.flat) and torch.equal(engs[0].opt_d.powers, e.opt_d.powers)
        assert engs[0].last_losses() == e.last_losses()


