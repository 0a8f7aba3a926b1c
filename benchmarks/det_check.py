"""Determinism probe: one training step of a fresh HIP engine (and of the fp32 PyTorch reference)
twice from the same init / z / batch; prints the max relative difference between the two runs per
model.  ``python -m benchmarks.det_check [--dtype fp32] [--graph 0]``"""
import argparse

import torch

from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
from distributed_tensorflow_for_dcgan_amd.engine.reference_step import ReferenceStep
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
from distributed_tensorflow_for_dcgan_amd.models.dcgan import DCGAN


def rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--graph", type=int, default=0)
    ap.add_argument("--B", type=int, default=16)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig()
    real = (torch.rand(a.B, 64, 64, 3, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(dev)
    runs, z = [], None
    for _ in range(3):
        eng = HipEngine(cfg, a.B, dev, graph=bool(a.graph), seed=3, dtype=a.dtype)
        eng.set_batch(real)
        eng.train_step()
        torch.cuda.synchronize()
        runs.append((eng.grad_g.flat.clone(), eng.grad_d.flat.clone()))
        z = eng.z.clone()
        del eng
    for i in (1, 2):
        print("engine run0 vs run%d: G %.3e D %.3e (bitwise %s)" % (i, rel(runs[i][0], runs[0][0]), rel(runs[i][1], runs[0][1]),
              torch.equal(runs[i][0], runs[0][0]) and torch.equal(runs[i][1], runs[0][1])))
    refs = []
    for _ in range(3):
        m = DCGAN(cfg, device=dev, seed=3)
        _, gd, gg = ReferenceStep(m).compute_grads(real, z)
        refs.append((gg.clone(), gd.clone()))
    for i in (1, 2):
        print("reference run0 vs run%d: G %.3e D %.3e" % (i, rel(refs[i][0], refs[0][0]), rel(refs[i][1], refs[0][1])))
    print("engine vs reference: G %.3e D %.3e" % (rel(runs[0][0], refs[0][0]), rel(runs[0][1], refs[0][1])))


if __name__ == "__main__":
    main()
