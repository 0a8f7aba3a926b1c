"""Study: the longest-phase-first igemm3 dispatch (DCGAN_IGEMM_LPT) only permutes workgroups, so two
engines that differ only in it must stay bit-identical step by step (eager, or graph replay with
LPT_EQ_GRAPH=1)."""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
dev = torch.device("cuda", 0)
GRAPH = os.environ.get("LPT_EQ_GRAPH", "0") == "1"
for size, c, B in ((28, 1, 64), (64, 3, 128), (64, 3, 32)):
    cfg = DCGANConfig(output_size=size, c_dim=c)
    real = (torch.rand(B, size, size, c, generator=torch.Generator().manual_seed(1)) * 2 - 1).to(dev)
    engs = []
    for f in ("0", "1"):
        os.environ["DCGAN_IGEMM_LPT"] = f
        e = HipEngine(cfg, B, dev, graph=GRAPH, seed=4)
        e.set_batch(real)
        engs.append(e)
    for step in range(4):
        for e in engs:
            e.train_step()
        torch.cuda.synchronize()
        a, b = engs
        bad = []
        for nm, x, y in (("g", a.model.g.flat, b.model.g.flat), ("d", a.model.d.flat, b.model.d.flat),
                         ("gg", a.grad_g.flat, b.grad_g.flat), ("gd", a.grad_d.flat, b.grad_d.flat)):
            if not torch.equal(x, y):
                bad.append((nm, float((x - y).abs().max())))
        print(size, B, "step", step, "losses equal", a.last_losses() == b.last_losses(), "diff", bad, flush=True)
