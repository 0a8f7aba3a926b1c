"""Checkpoint (TF V2 bundle + index file), resume exactness, event files, PNG grids."""
import os
import struct

import numpy as np
import pytest
import torch

from distributed_tensorflow_for_dcgan_amd.ckpt import checkpoint as CK, tf_bundle as TB
from distributed_tensorflow_for_dcgan_amd.engine.factory import ReferenceEngine
from distributed_tensorflow_for_dcgan_amd.models.config import DCGANConfig
from distributed_tensorflow_for_dcgan_amd.obs import events as EV, images as IM


def test_bundle_roundtrip_many_tensors(tmp_path):
    rng = np.random.RandomState(0)
    t = {"a/b": rng.randn(3, 4).astype(np.float32), "Variable": np.array(7, np.int32),
         "z": rng.randn(5).astype(np.float64), "beta1_power": np.array(0.25, np.float32)}
    for i in range(300):  # several data blocks / restart intervals
        t["layer_%03d/w" % i] = rng.randn(2, 3).astype(np.float32)
    prefix = str(tmp_path / "model.ckpt-7")
    TB.write_bundle(prefix, t)
    back = TB.read_bundle(prefix)
    assert set(back) == set(t)
    for k in t:
        assert back[k].dtype == t[k].dtype and back[k].shape == t[k].shape
        assert np.array_equal(back[k], t[k])
    table = TB.read_table(prefix + ".index")
    assert list(table)[0] == b"" and list(table) == sorted(table)
    raw = open(prefix + ".index", "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == TB.MAGIC


def test_bundle_small_blocks_and_corruption(tmp_path):
    prefix = str(tmp_path / "m")
    t = {"k%04d" % i: np.full((3,), i, np.float32) for i in range(100)}
    # force many blocks
    tw = TB.TableWriter(prefix + ".tmpidx", block_size=64)
    for k in sorted(t):
        tw.add(k.encode(), b"v" + k.encode())
    tw.close()
    tab = TB.read_table(prefix + ".tmpidx")
    assert len(tab) == 100 and tab[b"k0042"] == b"vk0042"
    TB.write_bundle(prefix, t)
    data = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    data[5] ^= 1
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(IOError):
        TB.read_bundle(prefix)


def test_snappy_decoder():
    # hand-built snappy stream: literal "abcd" + copy(offset 4, len 8) -> "abcdabcdabcd"
    comp = bytes([12]) + bytes([(4 - 1) << 2]) + b"abcd" + bytes([((8 - 4) << 2) | 1, 4])
    assert TB._snappy_decompress(comp) == b"abcdabcdabcd"


def test_index_file_roundtrip(tmp_path):
    CK.write_index(str(tmp_path), "model.ckpt-20", ["model.ckpt-10", "model.ckpt-20"])
    st = CK.read_index(str(tmp_path))
    assert st["model_checkpoint_path"] == "model.ckpt-20"
    assert st["all_model_checkpoint_paths"] == ["model.ckpt-10", "model.ckpt-20"]
    assert CK.latest_checkpoint(str(tmp_path)) is None  # files do not exist


def _engine(seed=0):
    cfg = DCGANConfig(output_size=28, c_dim=1)
    e = ReferenceEngine(cfg, 4, torch.device("cpu"), seed=seed, z_seed=11)
    return e


def _batches(n):
    g = torch.Generator().manual_seed(5)
    return [torch.rand(4, 28, 28, 1, generator=g) * 2 - 1 for _ in range(n)]


def test_resume_is_exact(tmp_path):
    """train 3 + save + restore into a fresh engine + train 2  ==  train 5 (optimiser state
    and BN averages included; z stream re-seeded identically after restore)."""
    data = _batches(5)
    a = _engine()
    for x in data:
        a.set_batch(x)
        a.train_step()
    b = _engine()
    for x in data[:3]:
        b.set_batch(x)
        b.train_step()
    mgr = CK.CheckpointManager(str(tmp_path), keep=2)
    mgr.save(b)
    zstate = b.z_gen.get_state()
    c = _engine(seed=123)  # different init: everything must come from the checkpoint
    info = mgr.restore_latest(c)
    assert info["global_step"] == 3 and info["adam_d"] and info["adam_g"]
    c.z_gen.set_state(zstate)
    for x in data[3:]:
        c.set_batch(x)
        c.train_step()
    assert c.global_step == 5
    assert torch.allclose(a.model.g.flat, c.model.g.flat, atol=1e-6)
    assert torch.allclose(a.model.d.flat, c.model.d.flat, atol=1e-6)
    assert torch.allclose(a.model.g_bn.flat, c.model.g_bn.flat, atol=1e-6)
    assert torch.allclose(a.opt_g.m.flat, c.opt_g.m.flat, atol=1e-7)
    # the moving-average update counts (zero-debias divisor) survive the restore as well
    assert torch.equal(a.model.g_bn.steps, c.model.g_bn.steps) and torch.equal(a.model.d_bn.steps, c.model.d_bn.steps)
    assert float(c.model.g_bn.steps[0]) > 0


def test_keep_last_n_and_reference_style_restore(tmp_path):
    e = _engine()
    mgr = CK.CheckpointManager(str(tmp_path), keep=2, save_secs=0)
    for s in (1, 2, 3):
        e.global_step = s
        mgr.save(e)
    st = CK.read_index(str(tmp_path))
    assert st["all_model_checkpoint_paths"] == ["model.ckpt-2", "model.ckpt-3"]
    assert not os.path.exists(str(tmp_path / "model.ckpt-1.index"))
    # a reference-style checkpoint: weights + EMA + global_step, no Adam slots
    sd = CK.collect_state(e)
    ref_sd = {k: v for k, v in sd.items() if "Adam" not in k and not k.startswith("beta") and "local_step" not in k}
    ref_sd["Variable"] = np.array(9, np.int32)
    TB.write_bundle(str(tmp_path / "model.ckpt-9"), ref_sd)
    CK.write_index(str(tmp_path), "model.ckpt-9", ["model.ckpt-9"])
    f = _engine(seed=5)
    info = mgr.restore_latest(f)
    assert info["global_step"] == 9 and info["adam_d"] is False
    assert torch.equal(f.model.d.flat, e.model.d.flat)
    assert float(f.opt_d.powers[0]) == 0.5
    # no saved update counts: one EMA update per synchronous step is assumed
    assert float(f.model.g_bn.steps[0]) == 9.0 and float(f.model.d_bn.steps[1]) == 9.0


def test_event_file_contents(tmp_path):
    w = EV.SummaryWriter(str(tmp_path))
    w.add_summary_values([EV.SummaryWriter.scalar("d_loss", 0.5),
                          EV.SummaryWriter.histogram("w", np.array([-1.0, 0.0, 0.5, 2.0])),
                          EV.SummaryWriter.image("G", np.random.rand(8, 8, 3))], step=3)
    w.close()
    ev = EV.read_events(w.path)
    assert ev[0]["file_version"] == "brain.Event:2"
    vals = {v["tag"]: v for v in ev[1]["values"]}
    assert ev[1]["step"] == 3 and abs(vals["d_loss"]["simple_value"] - 0.5) < 1e-7
    h = vals["w"]["histo"]
    assert struct.unpack("<d", h[3][0])[0] == 4.0  # num
    counts = np.frombuffer(h[7][0], "<f8")
    assert counts.sum() == 4
    img = vals["G"]["image"]
    assert img[1][0] == 8 and img[4][0][:8] == b"\x89PNG\r\n\x1a\n"


def test_histogram_buckets_match_tf_defaults():
    b = EV._default_buckets()
    assert b[len(b) // 2] == 0.0 and abs(b[len(b) // 2 + 1] - 1e-12) < 1e-24
    assert len(b) == 1551  # -DBL_MAX, 774 negative, 0, 774 positive, DBL_MAX


def test_png_and_grid(tmp_path):
    from PIL import Image
    imgs = np.random.uniform(-1, 1, (64, 6, 6, 3)).astype(np.float32)
    p = str(tmp_path / "g.png")
    IM.save_images(imgs, (8, 8), p)
    im = np.asarray(Image.open(p))
    assert im.shape == (48, 48, 3)
    gray = np.random.uniform(-1, 1, (4, 5, 5, 1))
    IM.save_images(gray, (2, 2), str(tmp_path / "m.png"))
    assert np.asarray(Image.open(str(tmp_path / "m.png"))).shape == (10, 10)
    raw = IM.encode_png(np.zeros((3, 4, 3), np.uint8))
    assert np.asarray(Image.open(__import__("io").BytesIO(raw))).shape == (3, 4, 3)
    assert IM.grid_size(64) == (8, 8)


def test_batch_dtype_follows_the_built_engine():
    """TFRecord batches are decoded into the compute dtype of the engine that was built -- never
    into bf16 for the fp32 reference engine (pipeline.batch_dtype)."""
    from distributed_tensorflow_for_dcgan_amd.data import pipeline as PL
    assert PL.batch_dtype("cuda", "bf16") == torch.bfloat16
    assert PL.batch_dtype("cuda", "fp16") == torch.float16
    assert PL.batch_dtype("cuda", "fp32") == torch.float32
    assert PL.batch_dtype("cuda", None) == torch.float32
    assert PL.batch_dtype("cpu", "bf16") == torch.float32
    assert ReferenceEngine.dtype_name == "fp32"
