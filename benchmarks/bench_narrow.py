"""Time the narrow (N=3) conv_transpose kernel at the step's shape (G's RGB layer / D layer-0
data gradient, B=128, 32x32x64 -> 64x64x3). DCGAN_NARROW_VALU=1 selects the v_dot2 kernel."""
import os

import torch

from distributed_tensorflow_for_dcgan_amd.ops import hip as H
from distributed_tensorflow_for_dcgan_amd.ops.hip import _p
from distributed_tensorflow_for_dcgan_amd.models.config import same_pads


def main():
    dev = torch.device("cuda", 0)
    B, Hi, C, Ho, N = 128, 32, 64, 64, 3
    x = (torch.randn(B, Hi, Hi, C, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(5, 5, N, C, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(B, Ho, Ho, N, device=dev, dtype=torch.bfloat16)
    prog = H.ext().Program(False)
    for _ in range(20):
        prog.narrow_deconv("narrow", _p(x), _p(w), 0, _p(y), B, Hi, Hi, C, Ho, Ho, N, same_pads(Ho)[0], 3, 0.2, 0)
    H.run(prog)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        H.run(prog)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 100
    print("narrow %s: %.2f us/launch" % ("valu" if os.environ.get("DCGAN_NARROW_VALU") else "mfma", us))
    # D layer 0 forward on the direct kernel (2B = 256 images, 64x64x3 -> 32x32x64, + bias + lrelu)
    xi = (torch.rand(256, 64, 64, 3, device=dev) * 2 - 1).to(torch.bfloat16)
    w0 = (torch.randn(5, 5, 3, 64, device=dev) * 0.05).to(torch.bfloat16)
    b0 = torch.zeros(64, device=dev)
    y0 = torch.empty(256, 32, 32, 64, device=dev, dtype=torch.bfloat16)
    prog = H.ext().Program(False)
    for _ in range(20):
        prog.conv3_direct("c3", _p(xi), _p(w0), _p(b0), _p(y0), 256, 64, 64, 3, 32, 32, 64, 1, 1, 2, 0.2, 0)
    H.run(prog)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        H.run(prog)
    e1.record()
    e1.synchronize()
    print("conv3 direct (D0 fwd, 2B=256): %.2f us/launch" % (e0.elapsed_time(e1) * 1000 / 100))


if __name__ == "__main__":
    main()
