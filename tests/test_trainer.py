"""End-to-end CLI runs on CPU: TFRecord data, log line, summaries, samples, checkpoint,
auto-resume, and kill/restart fault injection."""
import glob
import os
import re
import subprocess
import sys

import numpy as np

from distributed_tensorflow_for_dcgan_amd.data import tfrecord as TR

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = re.compile(r"^Epoch: \[\s*\d+\] step: \[\s*\d+\] time: \d+\.\d{4}, d_loss: -?\d+\.\d{8}, g_loss: -?\d+\.\d{8}")


def _run(args, env_extra=None, cwd=None):
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "image_train.py")] + args, env=env, cwd=cwd,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    return p.returncode, p.stdout


def _dataset(d, n=48, hw=28, c=1):
    os.makedirs(d, exist_ok=True)
    rng = np.random.RandomState(0)
    for f in range(3):
        TR.write_image_records(os.path.join(d, "train-%d.tfrecords" % f), rng.uniform(-1, 1, (n // 3, hw, hw, c)))


def test_train_from_tfrecords_and_resume(tmp_path):
    data = str(tmp_path / "train")
    _dataset(data)
    common = ["--data_dir=%s" % data, "--output_size=28", "--c_dim=1", "--batch_size=8", "--device=cpu",
              "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "samples"),
              "--shuffle_buffer=16", "--loader_threads=2", "--save_summaries_secs=0", "--sample_image_dir=nonexist"]
    rc, out = _run(common + ["--max_steps=4"])
    assert rc == 0, out
    lines = [l for l in out.splitlines() if l.startswith("Epoch:")]
    assert len(lines) == 4 and all(LINE.match(l) for l in lines), lines
    assert "load failed!!" in out and "[Sample] d_loss:" in out
    assert os.path.exists(tmp_path / "ck" / "checkpoint")
    assert glob.glob(str(tmp_path / "ck" / "events.out.tfevents.*"))
    assert os.path.exists(tmp_path / "samples" / "train_00_0001.png")
    # 48 examples / batch 8 -> 6 steps per epoch; --epoch=1 stops at global step 6
    rc, out = _run(common + ["--epoch=1"])
    assert rc == 0, out
    assert "load success!" in out and "global_step 4" in out
    steps = [int(re.search(r"step: \[\s*(\d+)\]", l).group(1)) for l in out.splitlines() if l.startswith("Epoch:")]
    assert steps == [5, 0]  # global steps 5 and 6 (6 % 6 == 0 -> epoch 1)
    assert os.path.exists(tmp_path / "ck" / "model.ckpt-6.index")


def test_fault_injection_and_restart(tmp_path):
    common = ["--synthetic", "--output_size=28", "--c_dim=1", "--batch_size=4", "--device=cpu",
              "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "s"),
              "--save_summaries_secs=1000", "--save_model_secs=1e-9", "--sample_every=0", "--max_steps=25"]
    rc, out = _run(common, env_extra={"DCGAN_FAULT_AT_STEP": "12"})
    assert rc == 3, out  # simulated crash after step 12 (checkpoints every SYNC_EVERY=10 steps)
    rc, out = _run(common)
    assert rc == 0, out
    assert "load success!" in out and "global_step 10" in out
    first = [l for l in out.splitlines() if l.startswith("Epoch:")][0]
    assert "step: [11]" in first
    assert os.path.exists(tmp_path / "ck" / "model.ckpt-25.index")


def test_sample_only_mode_and_visualize(tmp_path):
    """--nois_train restores the newest checkpoint and only samples (+ --visualize sweeps);
    without a checkpoint it refuses. The reference default (is_train unset) still trains."""
    common = ["--synthetic", "--output_size=28", "--c_dim=1", "--batch_size=8", "--device=cpu",
              "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "s"),
              "--save_summaries_secs=1000", "--sample_every=0"]
    rc, out = _run(common + ["--nois_train"])
    assert rc != 0 and "train a model first" in out
    rc, out = _run(common + ["--max_steps=2"])
    assert rc == 0 and len([l for l in out.splitlines() if l.startswith("Epoch:")]) == 2, out
    rc, out = _run(common + ["--is_train=false", "--visualize", "--num_samples=16"])
    assert rc == 0, out
    assert "[Test] wrote 16 samples" in out and not [l for l in out.splitlines() if l.startswith("Epoch:")]
    assert os.path.exists(tmp_path / "s" / "test_000002.png")
    assert os.path.exists(tmp_path / "s" / "test_arange_0.png") and os.path.exists(tmp_path / "s" / "test_interp.png")


def test_device_cache_source_and_timing_flags(tmp_path):
    data = str(tmp_path / "train")
    _dataset(data, n=48)
    rc, out = _run(["--data_dir=%s" % data, "--output_size=28", "--c_dim=1", "--batch_size=8", "--device=cpu",
                    "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "s"),
                    "--cache_on_device", "--timing", "--save_summaries_secs=1000", "--sample_every=0",
                    "--max_steps=3", "--loader_threads=2"])
    assert rc == 0, out
    assert len([l for l in out.splitlines() if l.startswith("Epoch:")]) == 3
