"""igemm5 diagnostics: per-row-block / per-channel-block error map of one conv launch."""
import sys
import torch
from distributed_tensorflow_for_dcgan_amd.ops import hip as h
from distributed_tensorflow_for_dcgan_amd.ops import reference as R

dev = "cuda"


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1).mul(scale).to(dev)


B, Hs, Ci, Co = [int(v) for v in sys.argv[1:5]] if len(sys.argv) > 4 else (4, 16, 128, 256)
cfgs = [int(c) for c in sys.argv[5].split(",")] if len(sys.argv) > 5 else [400]
x = rnd(B, Hs, Hs, Ci, seed=90).to(torch.bfloat16)
w = rnd(5, 5, Ci, Co, scale=0.05, seed=91).to(torch.bfloat16)
ref = R.conv2d_same(x.float(), w.float()).reshape(-1, Co)
for bkn in (0, 1):
    wp = w.reshape(25, Ci, Co).contiguous() if bkn else h.pack_conv_weight(w.float(), "conv", "fwd")
    for cfg in cfgs:
        for sp in (1, 3):
            y = h.conv2d_same(x, wp, Co, out_f32=True, cfg=cfg, bkn=bool(bkn), splits=sp).reshape(-1, Co)
            torch.cuda.synchronize()
            err = (y - ref).abs()
            M = err.shape[0]
            rows = err.reshape(-1, 16, Co).amax(dim=(1, 2))
            cols = err.amax(0).reshape(-1, 16).amax(1)
            print("cfg %d bkn %d sp %d max %.3e | bad 16-row blocks %s | bad 16-col blocks %s" % (
                cfg, bkn, sp, err.max().item(), (rows > 0.05).nonzero().flatten().tolist()[:40],
                (cols > 0.05).nonzero().flatten().tolist()[:40]))
