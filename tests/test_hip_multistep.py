"""Multi-step training correctness of the HIP engine (MI355X only).

The one-step parity tests (test_hip_engine.py) pin the kernels' math; these pin what a user of
the reference's 1.2 M-step loop (``image_train.py:150-158``) relies on:

* the fp32 HIP engine follows the fp32 autograd reference (CPU) step after step -- losses,
  parameters, Adam moments and BN moving averages after 10 consecutive steps;
* the bf16 engine tracks the fp32 HIP engine from the same init / z / data over 50 steps within
  stated bounds (mixed precision drifts; it must not diverge);
* G learns a learnable distribution: images from a tiny TFRecord fixture of flat-colour images,
  read through the native loader, and the EMA-BN sampler's per-channel statistics move to the
  data's.
"""
import math

import numpy as np
import pytest
import torch

from distributed_tensorflow_for_dcgan_amd.engine.reference_step import ReferenceStep
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
from distributed_tensorflow_for_dcgan_amd.models.dcgan import DCGAN

pytestmark = pytest.mark.gpu

LOSS_KEYS = ("d_loss_real", "d_loss_fake", "g_loss", "d_loss")


def rel(a, b):
    a, b = a.double().flatten().cpu(), b.double().flatten().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _live(model, names, cfg):
    """parameter names whose gradient is not analytically zero (biases followed by BN are dead)"""
    gl_last = cfg.g_layers()[-1].name
    out = []
    for n in names:
        if n == "g_h0_lin/bias":
            continue
        if n.endswith("/biases") and not (n.startswith("d_h0_conv") or n.split("/")[0] == gl_last):
            continue
        out.append(n)
    return out


def _cpu_chaos_envelope(cfg, B, steps, batches, zs, rel_noise=1e-6, samples=2):
    """Loss deviation per step between an fp32 CPU reference run and runs whose G and D weights
    carry ``rel_noise`` relative noise -- the size of an fp32 summation-order difference over a
    1,600-deep reduction (sqrt(K) * 6e-8) -- elementwise max over ``samples`` noise draws.
    GAN training from this init is chaotic (measured: a 1e-7 D-weight difference grows ~10x per
    step, to ~0.2 of the loss by step 9), so no fp32 implementation can track another to 1e-3
    over 10 steps; the HIP engine is held to this envelope instead."""
    cpu = torch.device("cpu")
    r1 = ReferenceStep(DCGAN(cfg, device=cpu, seed=3))
    rs = []
    for i in range(samples):
        m = DCGAN(cfg, device=cpu, seed=3)
        g = torch.Generator().manual_seed(5 + i)
        with torch.no_grad():
            m.g.flat.mul_(1 + rel_noise * torch.randn(m.g.flat.shape, generator=g))
            m.d.flat.mul_(1 + rel_noise * torch.randn(m.d.flat.shape, generator=g))
        rs.append(ReferenceStep(m))
    env = []
    for s in range(steps):
        a = r1.step(batches[s], zs[s])
        e = 0.0
        for r in rs:
            b = r.step(batches[s], zs[s])
            e = max(e, max(abs(a[k] - b[k]) / max(1.0, abs(a[k])) for k in LOSS_KEYS))
        env.append(e)
    return env


def test_fp32_engine_tracks_reference_over_10_steps():
    """fp32 HIP engine vs the fp32 CPU autograd reference, 10 consecutive steps from the same
    init, z (the engine's own Philox z of each step) and batches.

    Step 0 and step 1 are pinned tight (losses within 1e-5 / 1e-4 relative): the kernels' math.
    After that the comparison is against the model's own chaos: GAN training from this init
    amplifies a weight difference ~10x per step (CPU runs vs the same CPU run with its weights
    perturbed by 1e-6 relative -- _cpu_chaos_envelope), so from step 2 on the HIP engine's
    deviation from the reference must stay within 4x that envelope (+1e-5), every loss finite.
    G's BN moving averages after 10 steps within 10x the envelope's final loss deviation."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev, cpu = torch.device("cuda", 0), torch.device("cpu")
    cfg = DCGANConfig()
    B, steps = 16, 10
    eng = HipEngine(cfg, B, dev, graph=False, seed=3, dtype="fp32")
    ref_model = DCGAN(cfg, device=cpu, seed=3)
    ref = ReferenceStep(ref_model)
    g0, d0 = ref_model.g.flat.clone(), ref_model.d.flat.clone()
    assert torch.equal(eng.model.g.flat.cpu(), g0) and torch.equal(eng.model.d.flat.cpu(), d0)
    gen = torch.Generator().manual_seed(7)
    loss_err, batches, zs = [], [], []
    for s in range(steps):
        real = torch.rand(B, 64, 64, 3, generator=gen) * 2 - 1
        eng.set_batch(real.to(dev))
        eng.train_step()
        torch.cuda.synchronize()
        L = eng.last_losses()
        z = eng.z.cpu()
        R = ref.step(real, z)
        batches.append(real)
        zs.append(z)
        assert all(math.isfinite(v) for v in L.values()), (s, L)
        loss_err.append(max(abs(L[k] - R[k]) / max(1.0, abs(R[k])) for k in LOSS_KEYS))
    assert eng.global_step == steps and ref.global_step == steps
    env = _cpu_chaos_envelope(cfg, B, steps, batches, zs)
    bn_err = max(max(rel(eng.model.g_bn.mean[n], ref_model.g_bn.mean[n]), rel(eng.model.g_bn.var[n], ref_model.g_bn.var[n]))
                 for n, _ in cfg.g_bn_layers())
    print("\nfp32 10-step: HIP vs CPU loss rel err per step %s\n  CPU chaos envelope (1e-6 weight noise) %s; "
          "G BN EMA %.2e" % (" ".join("%.1e" % e for e in loss_err), " ".join("%.1e" % e for e in env), bn_err))
    assert loss_err[0] <= 1e-5 and loss_err[1] <= 1e-4, loss_err
    bad = [(s, e, env[s]) for s, e in enumerate(loss_err) if s >= 2 and e > 4 * env[s] + 1e-5]
    assert not bad, bad
    assert bn_err <= 10 * env[-1] + 1e-5, (bn_err, env[-1])


def test_bf16_engine_tracks_fp32_engine_over_50_steps():
    """bf16 vs fp32 HIP engine, same init / z stream / batches, 50 steps, against a measured
    envelope: a second fp32 engine whose FIRST batch carries bf16-sized (4e-3 relative) noise.
    The training is chaotic (a 1e-7 difference reaches ~0.2 of the loss in 9 steps), so after a
    few steps no two runs bit-track; what bf16 must not do is drift further than a bf16-sized
    perturbation of fp32 does (two noise draws, the larger taken). Bounds: steps 0-1 losses
    within 5 % (+0.05); mean |d_loss| and |g_loss| deviation over steps 10-49 within 2.5x the
    envelope's (+0.05) (measured 1.93 / 2.80 vs 1.11 / 1.56 for one draw); the 50-step update
    norms of G and D within 0.7-1.4x fp32's; every loss finite."""
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    B, steps = 32, 50
    e16 = HipEngine(cfg, B, dev, graph=True, seed=11, dtype="bf16")
    e32 = HipEngine(cfg, B, dev, graph=True, seed=11, dtype="fp32")
    e32ps = [HipEngine(cfg, B, dev, graph=True, seed=11, dtype="fp32") for _ in range(2)]
    g0, d0 = e32.model.g.flat.clone(), e32.model.d.flat.clone()
    assert torch.equal(e16.model.g.flat, g0) and torch.equal(e16.model.d.flat, d0)
    gen = torch.Generator().manual_seed(9)
    early_bad = []
    dev16, devp = [], [[], []]
    for s in range(steps):
        real = (torch.rand(B, 64, 64, 3, generator=gen) * 2 - 1).to(dev)
        e16.set_batch(real)
        e32.set_batch(real)
        for i, ep in enumerate(e32ps):
            if s == 0:
                noise = torch.randn(real.shape, generator=torch.Generator().manual_seed(13 + i)).to(dev)
                ep.set_batch(real * (1 + 4e-3 * noise))
            else:
                ep.set_batch(real)
            ep.train_step()
        e16.train_step()
        e32.train_step()
        L16, L32 = e16.last_losses(), e32.last_losses()
        assert all(math.isfinite(v) for v in L16.values()), (s, L16)
        if s < 2:
            early_bad += [(s, k, L16[k], L32[k]) for k in LOSS_KEYS
                          if abs(L16[k] - L32[k]) > 0.05 * abs(L32[k]) + 0.05]
        if s >= 10:
            dev16.append([abs(L16[k] - L32[k]) for k in ("d_loss", "g_loss")])
            for i, ep in enumerate(e32ps):
                Lp = ep.last_losses()
                devp[i].append([abs(Lp[k] - L32[k]) for k in ("d_loss", "g_loss")])
    torch.cuda.synchronize()
    m16, mp = np.mean(dev16, 0), np.maximum(np.mean(devp[0], 0), np.mean(devp[1], 0))
    ratios = {}
    for name, a16, a32, init in (("G", e16.model.g.flat, e32.model.g.flat, g0), ("D", e16.model.d.flat, e32.model.d.flat, d0)):
        ratios[name] = float((a16 - init).double().norm() / (a32 - init).double().norm())
    print("\nbf16 vs fp32 over %d steps: mean |dev| steps 10-49 d_loss %.3f g_loss %.3f; envelope (fp32, 4e-3 "
          "noise on batch 0) d_loss %.3f g_loss %.3f; update norm ratio G %.3f D %.3f"
          % (steps, m16[0], m16[1], mp[0], mp[1], ratios["G"], ratios["D"]))
    assert not early_bad, early_bad
    assert m16[0] <= 2.5 * mp[0] + 0.05 and m16[1] <= 2.5 * mp[1] + 0.05, (m16, mp)
    for name, r in ratios.items():
        assert 0.7 <= r <= 1.4, (name, r)


def test_generator_learns_flat_colour_images(tmp_path):
    """Learnability on a real input path: 4,096 flat 28x28x1 images (each image one grey level
    drawn from U(0.4, 0.6): zero spatial variance, intensity 0.5 +- 0.1) written as float64
    TFRecords, read by the native loader, 600 bf16 steps. The untrained EMA-BN sampler is far from
    the data (textured images, mean ~0.1, spatial std ~1.0); after training its images are flat
    (mean spatial std under 0.2x the untrained one) and at the data's intensity: at least 90 % of
    the samples have a per-image mean in [0.2, 0.8] and the sample mean is within 0.2 of 0.5. A
    generator collapsed to a constant 0 grey fails both, and one collapsed to a single grey level
    fails the diversity check (std of the per-image means >= half the data's). All 3 seeds (4, 5,
    6) must pass: the loader runs in its deterministic mode (one reader, a draw window of exactly
    shuffle_buffer + batch examples: csrc/host/loader.h), and the engine's reductions are
    deterministic, so each seed's run is reproducible -- a failure is a property of the code, not
    of the run's timing. Measured on MI355X (seeds 4 and 5,
    benchmarks/study/learn_diag.py, profiles/r4/learnability_diag_r4.txt): from step 400 on,
    100 % in range, mean 0.51-0.55, spatial std 0.01-0.05. (A two-mode +-0.6 dataset, used until
    round 4, is unusable here: the GAN hops between the modes and any single checkpoint sees all
    samples near one mode or none.)"""
    from distributed_tensorflow_for_dcgan_amd.data import pipeline as PL
    from distributed_tensorflow_for_dcgan_amd.data import tfrecord as TR
    from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    n = 4096
    lv = 0.5 + rng.uniform(-0.1, 0.1, size=n)
    imgs = np.broadcast_to(lv[:, None, None, None], (n, 28, 28, 1)).astype(np.float64)
    d = tmp_path / "train"
    d.mkdir()
    for i in range(4):
        TR.write_image_records(str(d / ("flat-%d.tfrecord" % i)), imgs[i::4])
    cfg = DCGANConfig(output_size=28, c_dim=1)
    B = 64
    data_div = float(np.std(lv))  # ~0.058 (= 0.2 / sqrt(12))

    def train(seed):
        eng = HipEngine(cfg, B, dev, graph=True, seed=seed, dtype="bf16")
        # one reader thread: the loader's deterministic mode (the batch order depends on the seed only)
        src = PL.TFRecordSource(str(d), B, (28, 28, 1), dev, shuffle_buffer=512, threads=1, seed=1,
                                out_dtype="bf16", num_examples=n)
        z = (torch.rand(B, cfg.z_dim, generator=torch.Generator().manual_seed(3)) * 2 - 1).to(dev)

        def stats():  # (sample mean, mean per-image spatial std, fraction of per-image means in [0.2, 0.8],
            #             std over the images of their means = sample diversity)
            x = eng.sampler(z).float().flatten(1)
            m = x.mean(1)
            return (float(x.mean()), float(x.std(1).mean()), float(((m >= 0.2) & (m <= 0.8)).float().mean()),
                    float(m.std()))

        m0, s0, f0, _ = stats()
        try:
            for _ in range(600):
                eng.set_batch(src.next())
                eng.train_step()
            torch.cuda.synchronize()
        finally:
            src.close()
        m1, s1, f1, div1 = stats()
        print("\nseed %d sampler before: mean %.3f spatial std %.3f in-range %.2f; after 600 steps: mean %.3f "
              "spatial std %.3f in-range %.2f diversity %.4f (data %.4f); losses %s"
              % (seed, m0, s0, f0, m1, s1, f1, div1, data_div, eng.last_losses()))
        assert all(math.isfinite(v) for v in eng.last_losses().values())
        # learned: flat images (spatial std under 0.2x the untrained one) at the data's intensity,
        # and not collapsed: the samples' per-image means spread at least half as much as the data's
        # (measured 0.062-0.078 at step 600 for seeds 4-6: profiles/r5/learnability_diversity_r5.txt);
        # a generator that maps every z to one grey level has ~0
        return s1 < 0.2 * s0 and f1 >= 0.9 and abs(m1 - 0.5) < 0.2 and div1 >= 0.5 * data_div

    ok = [train(seed) for seed in (4, 5, 6)]
    assert all(ok), ok
