"""Host time to issue one training step (eager C++ replay) vs the GPU time of a step: is the step
host-bound anywhere? Prints the host-side issue time of single steps issued onto an idle GPU, and
the steady-state host/GPU rates over 200 back-to-back steps."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    graph = os.environ.get("HOST_ISSUE_GRAPH", "0") == "1"
    eng = HipEngine(DCGANConfig(), 128, dev, graph=graph, seed=0)
    eng.set_batch(torch.rand(128, 64, 64, 3, device=dev) * 2 - 1)
    for _ in range(10):
        eng.train_step()
    torch.cuda.synchronize()
    single = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.train_step()
        single.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    single.sort()
    t0 = time.perf_counter()
    for _ in range(200):
        eng.train_step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("graph=%d host issue of one step on an idle GPU: median %.0f us (min %.0f, max %.0f)"
          % (graph, single[10], single[0], single[-1]))
    print("graph=%d 200 steps: host issue %.0f us/step, GPU %.0f us/step (host done %.1f ms before the GPU)"
          % (graph, (t1 - t0) / 200 * 1e6, (t2 - t0) / 200 * 1e6, (t2 - t1) * 1e3))


if __name__ == "__main__":
    main()
