"""The HIP engine inside the full framework on an MI355X: checkpoint / resume through the TF
V2 bundle layout is bit-exact (weights, Adam slots, beta powers, BN moving averages, global
step, the bf16 weight mirrors refreshed on load), and the reference CLI (image_train.py) trains
from TFRecords on the HIP engine with the reference log line, checkpoints, samples and
TensorBoard events."""
import glob
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = re.compile(r"^Epoch: \[\s*\d+\] step: \[\s*\d+\] time: \d+\.\d{4}, d_loss: -?\d+\.\d{8}, g_loss: -?\d+\.\d{8}")


def _engine(graph=True):
    from distributed_tensorflow_for_dcgan_amd.engine.factory import build_engine
    from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
    eng = build_engine(DCGANConfig(output_size=64, c_dim=3), 16, torch.device("cuda", 0), engine="hip", seed=11,
                       graph=graph)
    real = torch.rand(16, 64, 64, 3, generator=torch.Generator().manual_seed(12)) * 2 - 1
    eng.set_batch(real.cuda())
    return eng


def _state(eng):
    torch.cuda.synchronize()
    return [t.detach().cpu().clone() for t in (eng.model.g.flat, eng.model.d.flat, eng.opt_g.m.flat, eng.opt_g.v.flat,
                                               eng.opt_d.m.flat, eng.opt_d.v.flat, eng.model.g_bn.flat,
                                               eng.model.d_bn.flat)]


def test_hip_checkpoint_resume_is_bit_exact(tmp_path):
    from distributed_tensorflow_for_dcgan_amd.ckpt.checkpoint import CheckpointManager
    ref = _engine()
    for _ in range(6):
        ref.train_step()
    want = _state(ref)
    assert ref.global_step == 6
    a = _engine()
    for _ in range(3):
        a.train_step()
    CheckpointManager(str(tmp_path)).save(a)
    del a
    b = _engine()  # fresh random init, then restore: the bf16 mirrors must be refreshed too
    info = CheckpointManager(str(tmp_path)).restore_latest(b)
    assert info["global_step"] == 3 and b.global_step == 3
    for _ in range(3):
        b.train_step()
    got = _state(b)
    assert b.global_step == 6
    for w, g in zip(want, got):
        assert torch.equal(w, g), (w - g).abs().max()


def _dataset(d, n=48, hw=64, c=3):
    from distributed_tensorflow_for_dcgan_amd.data import tfrecord as TR
    os.makedirs(d, exist_ok=True)
    rng = np.random.RandomState(0)
    for f in range(3):
        TR.write_image_records(os.path.join(d, "train-%d.tfrecords" % f), rng.uniform(-1, 1, (n // 3, hw, hw, c)))


def test_image_train_cli_on_hip_engine(tmp_path):
    data = str(tmp_path / "train")
    _dataset(data)
    args = ["--data_dir=%s" % data, "--batch_size=8", "--device=cuda", "--engine=hip",
            "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "samples"),
            "--shuffle_buffer=16", "--loader_threads=2", "--save_summaries_secs=0", "--sample_image_dir=nonexist",
            "--max_steps=3"]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "image_train.py")] + args, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    out = p.stdout
    assert p.returncode == 0, out[-3000:]
    lines = [l for l in out.splitlines() if l.startswith("Epoch:")]
    assert len(lines) == 3 and all(LINE.match(l) for l in lines), lines
    assert "[Sample] d_loss:" in out
    assert os.path.exists(tmp_path / "ck" / "checkpoint")
    assert glob.glob(str(tmp_path / "ck" / "model.ckpt-3.index"))
    assert glob.glob(str(tmp_path / "ck" / "events.out.tfevents.*"))
    assert glob.glob(str(tmp_path / "samples" / "*.png"))
