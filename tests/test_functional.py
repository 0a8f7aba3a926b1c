"""ops.functional: autograd conv / conv_transpose on the HIP kernels vs the PyTorch fp32
reference ops (ops.reference) on the same bf16-rounded operands -- forward, input gradient,
weight gradient and bias gradient, including the narrow 3-channel cases (im2col paths)."""
import pytest
import torch

from distributed_tensorflow_for_dcgan_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _close(a, b, rel, name):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= rel * scale, "%s: err %.3e scale %.3e" % (name, err, scale)


def _ref_grads(fn, x, w, b, dy):
    x = x.detach().float().requires_grad_(True)
    w = w.detach().float().requires_grad_(True)
    b = b.detach().float().requires_grad_(True)
    y = fn(x, w, b)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), dy.float())
    return y, gx, gw, gb


@pytest.mark.parametrize("B,Hs,ci,co", [(4, 16, 64, 128), (2, 64, 3, 64), (3, 8, 128, 256)])
def test_conv2d_same_autograd(B, Hs, ci, co):
    from distributed_tensorflow_for_dcgan_amd.ops import functional as F
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(B, Hs, Hs, ci, generator=g) * 2 - 1).cuda().to(torch.bfloat16)
    w = (torch.randn(5, 5, ci, co, generator=g) * 0.05).cuda().to(torch.bfloat16).float().requires_grad_(True)
    b = (torch.randn(co, generator=g) * 0.1).cuda().requires_grad_(True)
    xr = x.float().requires_grad_(True)
    y = F.conv2d_same(xr, w, b)
    dy = (torch.rand_like(y.float()) - 0.5).to(torch.bfloat16)
    gx, gw, gb = torch.autograd.grad(y, (xr, w, b), dy)
    ry, rgx, rgw, rgb = _ref_grads(lambda a, c, d: R.conv2d_same(a, c, d), x, w, b, dy)
    _close(y, ry, 1.5e-2, "fwd")
    _close(gx, rgx, 1.5e-2, "dx")
    _close(gw, rgw, 2e-3, "dw")
    _close(gb, rgb, 2e-3, "db")


@pytest.mark.parametrize("B,Hi,Ho,ci,co", [(4, 8, 16, 128, 64), (2, 32, 64, 64, 3), (2, 4, 7, 64, 64)])
def test_conv2d_transpose_same_autograd(B, Hi, Ho, ci, co):
    from distributed_tensorflow_for_dcgan_amd.ops import functional as F
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(B, Hi, Hi, ci, generator=g) * 2 - 1).cuda().to(torch.bfloat16)
    w = (torch.randn(5, 5, co, ci, generator=g) * 0.05).cuda().to(torch.bfloat16).float().requires_grad_(True)
    b = (torch.randn(co, generator=g) * 0.1).cuda().requires_grad_(True)
    xr = x.float().requires_grad_(True)
    y = F.conv2d_transpose_same(xr, w, (Ho, Ho), b)
    dy = (torch.rand_like(y.float()) - 0.5).to(torch.bfloat16)
    gx, gw, gb = torch.autograd.grad(y, (xr, w, b), dy)
    ry, rgx, rgw, rgb = _ref_grads(lambda a, c, d: R.conv2d_transpose_same(a, c, (Ho, Ho), d), x, w, b, dy)
    _close(y, ry, 1.5e-2, "fwd")
    _close(gx, rgx, 1.5e-2, "dx")
    _close(gw, rgw, 2e-3, "dw")
    _close(gb, rgb, 2e-3, "db")


def test_modules_train_a_step():
    from distributed_tensorflow_for_dcgan_amd.ops import functional as F
    torch.manual_seed(0)
    conv = F.Conv2dSame(64, 128, device="cuda")
    deconv = F.ConvTranspose2dSame(128, 64, device="cuda")
    opt = torch.optim.Adam(list(conv.parameters()) + list(deconv.parameters()), lr=1e-3)
    x = torch.rand(4, 16, 16, 64, device="cuda") * 2 - 1
    losses = []
    for _ in range(5):
        y = deconv(torch.relu(conv(x).float()), (16, 16))
        loss = (y.float() - x).pow(2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
