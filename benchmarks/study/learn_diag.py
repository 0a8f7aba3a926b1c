"""Learnability diagnostics for tests/test_hip_multistep.py: per-image mean statistics of the
EMA sampler and of the last training batch's fakes at checkpoints, for a two-mode (+-0.6) and a
one-mode (0.5 +- 0.1) flat-grey dataset. `div` = std over the sampler's images of their means
(sample diversity; the one-mode data's own is 0.2 / sqrt(12) = 0.058), so a generator that maps
every z to one grey level shows div ~ 0.

    python benchmarks/study/learn_diag.py [one|two ...] [--seeds 4,5] [--steps 200,400,600]"""
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, ".")
from distributed_tensorflow_for_dcgan_amd.data import pipeline as PL  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.data import tfrecord as TR  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig  # noqa: E402


def run(kind, seed, steps=(200, 400, 600, 800, 1000, 1200)):
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    n = 4096
    lv = rng.choice(np.array([-0.6, 0.6]), size=n) if kind == "two" else 0.5 + rng.uniform(-0.1, 0.1, size=n)
    imgs = np.broadcast_to(lv[:, None, None, None], (n, 28, 28, 1)).astype(np.float64)
    with tempfile.TemporaryDirectory() as d:
        for i in range(4):
            TR.write_image_records("%s/flat-%d.tfrecord" % (d, i), imgs[i::4])
        cfg = DCGANConfig(output_size=28, c_dim=1)
        B = 64
        eng = HipEngine(cfg, B, dev, graph=True, seed=seed, dtype="bf16")
        src = PL.TFRecordSource(d, B, (28, 28, 1), dev, shuffle_buffer=512, threads=4, seed=1, out_dtype="bf16",
                                num_examples=n)
        z = (torch.rand(B, cfg.z_dim, generator=torch.Generator().manual_seed(3)) * 2 - 1).to(dev)
        done = 0
        try:
            for s in steps:
                while done < s:
                    eng.set_batch(src.next())
                    eng.train_step()
                    done += 1
                x = eng.sampler(z).float().flatten(1)
                m = x.mean(1)
                f = eng.fake.float().flatten(1).mean(1)
                print("%s seed %d step %4d  sampler: mean %+.3f near(|m|>=.3) %.2f in[.2,.8] %.2f std %.3f div %.4f | "
                      "train fakes: mean %+.3f near %.2f in[.2,.8] %.2f div %.4f" % (
                          kind, seed, s, m.mean(), (m.abs() >= 0.3).float().mean(), ((m > 0.2) & (m < 0.8)).float().mean(),
                          x.std(1).mean(), m.std(), f.mean(), (f.abs() >= 0.3).float().mean(),
                          ((f > 0.2) & (f < 0.8)).float().mean(), f.std()), flush=True)
        finally:
            src.close()


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("kinds", nargs="*", default=["two", "one"])
    ap.add_argument("--seeds", default="4,5")
    ap.add_argument("--steps", default="200,400,600,800,1000,1200")
    a = ap.parse_args()
    for kind in a.kinds:
        for seed in (int(v) for v in a.seeds.split(",")):
            run(kind, seed, tuple(int(v) for v in a.steps.split(",")))
