"""TF semantics of the reference ops on CPU, in float64."""
import math

import numpy as np
import pytest
import torch

from distributed_tensorflow_for_dcgan_amd.models.config import same_out, same_pads
from distributed_tensorflow_for_dcgan_amd.ops import reference as R


@pytest.fixture(autouse=True)
def _float64():
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    yield
    torch.set_default_dtype(old)


def naive_conv_same(x, w, stride=2):
    """Direct loop implementation of tf.nn.conv2d(padding='SAME') for NHWC/HWIO."""
    B, H, W, Ci = x.shape
    kh, kw, _, Co = w.shape
    Ho, Wo = same_out(H, stride), same_out(W, stride)
    ply, plx = same_pads(H, kh, stride)[0], same_pads(W, kw, stride)[0]
    y = torch.zeros(B, Ho, Wo, Co)
    for oy in range(Ho):
        for ox in range(Wo):
            for ky in range(kh):
                for kx in range(kw):
                    iy, ix = oy * stride + ky - ply, ox * stride + kx - plx
                    if 0 <= iy < H and 0 <= ix < W:
                        y[:, oy, ox, :] += x[:, iy, ix, :] @ w[ky, kx]
    return y


@pytest.mark.parametrize("n,expect", [(64, (1, 2)), (32, (1, 2)), (8, (1, 2)), (28, (1, 2)), (14, (1, 2)),
                                      (7, (2, 2)), (4, (1, 2))])
def test_same_pads(n, expect):
    assert same_pads(n) == expect


@pytest.mark.parametrize("H", [8, 7, 14, 5])
def test_conv2d_same_matches_loop(H):
    g = torch.Generator().manual_seed(H)
    x = torch.randn(2, H, H, 3, generator=g)
    w = torch.randn(5, 5, 3, 4, generator=g)
    assert torch.allclose(R.conv2d_same(x, w), naive_conv_same(x, w), atol=1e-10)


def test_pytorch_symmetric_padding_is_different():
    x = torch.randn(1, 8, 8, 2)
    w = torch.randn(5, 5, 2, 2)
    sym = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), stride=2, padding=2)
    assert (sym.permute(0, 2, 3, 1) - R.conv2d_same(x, w)).abs().max() > 1e-3


@pytest.mark.parametrize("Hi,Ho", [(4, 8), (8, 16), (4, 7), (2, 4), (7, 14)])
def test_conv_transpose_is_exact_adjoint(Hi, Ho):
    """<conv(y), x> == <y, conv_T(x)> for the TF-SAME pair."""
    g = torch.Generator().manual_seed(Hi * 31 + Ho)
    w = torch.randn(5, 5, 3, 4, generator=g)  # deconv [kh,kw,out=3,in=4]; conv HWIO [.., in=3, out=4]
    x = torch.randn(2, Hi, Hi, 4, generator=g)
    y = torch.randn(2, Ho, Ho, 3, generator=g)
    lhs = (R.conv2d_same(y, w) * x).sum()
    rhs = (y * R.conv2d_transpose_same(x, w, (Ho, Ho))).sum()
    assert abs(float(lhs - rhs)) < 1e-9 * max(1.0, abs(float(lhs)))
    assert R.conv2d_same(y, w).shape[1] == Hi


def test_batch_norm_tf_semantics_and_groups():
    x = torch.randn(6, 4, 4, 5) * 3 + 1
    beta, gamma = torch.randn(5), torch.rand(5) + 0.5
    m, v = R.moments(x)
    assert torch.allclose(m[0], x.reshape(-1, 5).mean(0))
    assert torch.allclose(v[0], x.reshape(-1, 5).var(0, unbiased=False))  # biased variance
    y = R.batch_norm(x, m[0], v[0], beta, gamma, 1e-5)
    assert torch.allclose(y, (x - m[0]) / torch.sqrt(v[0] + 1e-5) * gamma + beta)
    mg, vg = R.moments(x, groups=2)
    yg = R.batch_norm(x, mg, vg, beta, gamma, 1e-5, groups=2)
    y0 = R.batch_norm(x[:3], *[t[0] for t in R.moments(x[:3])], beta, gamma, 1e-5)
    assert torch.allclose(yg[:3], y0)


def test_bce_matches_tf_formula_and_is_stable():
    x = torch.tensor([-100.0, -3.0, 0.0, 2.5, 100.0])
    t = torch.tensor([1.0, 0.0, 1.0, 1.0, 0.0])
    got = R.sigmoid_cross_entropy_with_logits(x, t)
    ref = -(t * torch.log(torch.sigmoid(x).clamp_min(1e-300)) + (1 - t) * torch.log((1 - torch.sigmoid(x)).clamp_min(1e-300)))
    assert torch.isfinite(got).all()
    assert torch.allclose(got[1:4], ref[1:4])
    assert abs(float(got[0]) - 100.0) < 1e-6 and abs(float(got[4]) - 100.0) < 1e-6
    dr, df, gl, dl = R.gan_losses(torch.tensor([0.3, -0.2]), torch.tensor([0.1, 0.4]))
    assert torch.allclose(dl, dr + df)


def test_lrelu_and_zero_fraction():
    x = torch.tensor([-2.0, 0.0, 3.0])
    assert torch.equal(R.lrelu(x), torch.tensor([-0.4, 0.0, 3.0]))
    assert float(R.zero_fraction(torch.tensor([0.0, 1.0, 0.0, 2.0]))) == 0.5


def test_tf_adam_epsilon_placement():
    """TF: w -= lr_t * m / (sqrt(v) + eps) with lr_t carrying the bias correction; differs from
    torch.optim.Adam for tiny gradients."""
    w = torch.zeros(3)
    g = torch.tensor([1e-9, 1e-3, 1.0])
    m, v = torch.zeros(3), torch.zeros(3)
    R.tf_adam_update(w, g, m, v, 0.5, 0.999, lr=2e-4, beta1=0.5)
    lr_t = 2e-4 * math.sqrt(1 - 0.999) / (1 - 0.5)
    exp = -lr_t * (0.5 * g) / (torch.sqrt(0.001 * g * g) + 1e-8)
    assert torch.allclose(w, exp)
    wt = torch.zeros(3, requires_grad=True)
    opt = torch.optim.Adam([wt], lr=2e-4, betas=(0.5, 0.999), eps=1e-8)
    wt.grad = g.clone()
    opt.step()
    assert abs(float(wt[0]) - float(w[0])) > 1e-6 * abs(float(w[0]))  # tiny-gradient regime differs
