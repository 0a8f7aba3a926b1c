"""Step time of successive HipEngine builds in ONE process (the in-situ tuner's situation).

Every build used to create fresh HIP streams; HIP assigns new streams to its few hardware queues
in turn, so some builds got the D-chain stream on the main stream's queue and ran ~28 % slower.
``DCGAN_FRESH_STREAMS=1`` restores per-engine streams for the A/B."""
import argparse
import gc
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_for_dcgan_amd.engine import hip_engine as HE  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--builds", type=int, default=12)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    fresh = os.environ.get("DCGAN_FRESH_STREAMS", "0") == "1"
    dev = torch.device("cuda", 0)
    cfg = DCGANConfig(output_size=64, c_dim=3)
    real = torch.rand(128, 64, 64, 3, device=dev) * 2 - 1
    out = []
    for b in range(a.builds):
        if fresh:
            HE._STREAMS.clear()
        eng = HE.HipEngine(cfg, 128, dev, dtype="bf16", seed=b, graph=False)
        eng.set_synthetic_batch(real)
        for _ in range(10):
            eng.train_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.train_step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        out.append(ms)
        print("build %2d: %.4f ms/step" % (b, ms), flush=True)
        del eng
        gc.collect()
    print("fresh_streams=%d  min %.4f  max %.4f  max/min %.3f" % (fresh, min(out), max(out), max(out) / min(out)))


if __name__ == "__main__":
    main()
