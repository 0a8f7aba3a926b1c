"""CLI flag parity with the reference's tf.app.flags (image_train.py:10-40)."""
import math

import pytest

from distributed_tensorflow_for_dcgan_amd.utils import flags as F

REF_DEFAULTS = {
    "epoch": 25, "learning_rate": 0.0002, "beta1": 0.5, "train_size": math.inf, "batch_size": 64,
    "image_size": 108, "output_size": 64, "c_dim": 3, "dataset": "celebA", "checkpoint_dir": "checkpoint",
    "sample_dir": "samples", "is_train": False, "is_crop": False, "visualize": False, "data_dir": "train",
    "sample_image_dir": "sample_data", "ps_hosts": "", "worker_hosts": "", "job_name": "", "task_index": 0,
    "log_device_placement": True, "save_summaries_secs": 10,
}


def test_all_reference_flags_with_defaults():
    fl = F.parse_flags([])
    assert len(F.REFERENCE_FLAGS) == 22
    for k, v in REF_DEFAULTS.items():
        assert getattr(fl, k) == v, k
    assert set(REF_DEFAULTS) <= set(fl.as_dict())
    assert fl.__getattr__("__flags")["batch_size"] == 64


def test_flag_syntax_variants():
    fl = F.parse_flags(["--batch_size=128", "--learning_rate", "0.001", "--is_crop", "--nolog_device_placement",
                        "--is_train=false", "--train_size=inf", "--dataset", "mnist"])
    assert fl.batch_size == 128 and fl.learning_rate == 0.001
    assert fl.is_crop is True and fl.log_device_placement is False and fl.is_train is False
    assert fl.train_size == math.inf and fl.dataset == "mnist"
    fl = F.parse_flags(["--is_train=1", "--visualize", "true"])
    assert fl.is_train is True and fl.visualize is True


def test_unknown_flag_rejected():
    with pytest.raises(SystemExit):
        F.parse_flags(["--no_such_flag=1"])


def test_cluster_mapping(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    fl = F.parse_flags(["--job_name=worker", "--task_index=1", "--worker_hosts=127.0.0.1:2222,127.0.0.1:2223",
                        "--ps_hosts=127.0.0.1:2221"])
    c = F.cluster_from_flags(fl)
    assert c["world_size"] == 2 and c["rank"] == 1 and c["master_port"] == 2222
    assert c["local_rank"] == 1  # second worker listed for this host -> second GPU
    fl2 = F.parse_flags(["--task_index=2", "--worker_hosts=hostA:1,hostB:1,hostA:2,hostB:2"])
    assert F.cluster_from_flags(fl2)["local_rank"] == 1
    fl3 = F.parse_flags(["--task_index=1", "--worker_hosts=hostA:1,hostB:1,hostA:2,hostB:2"])
    assert F.cluster_from_flags(fl3)["local_rank"] == 0
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "3")
    c = F.cluster_from_flags(fl)
    assert (c["rank"], c["world_size"], c["source"]) == (3, 8, "env")
    monkeypatch.delenv("RANK")
    monkeypatch.delenv("WORLD_SIZE")
    with pytest.raises(ValueError):
        F.cluster_from_flags(F.parse_flags(["--task_index=5", "--worker_hosts=a:1,b:2"]))


def test_ps_role_exits_cleanly(tmp_path, capsys):
    from distributed_tensorflow_for_dcgan_amd.train.trainer import run
    fl = F.parse_flags(["--job_name=ps", "--checkpoint_dir=%s" % (tmp_path / "c")])
    assert run(fl) == 0
    assert "no parameter server" in capsys.readouterr().out


def test_bad_job_name():
    from distributed_tensorflow_for_dcgan_amd.train.trainer import run
    with pytest.raises(SystemExit):
        run(F.parse_flags(["--job_name=chief"]))


def test_dataset_preset(tmp_path, monkeypatch):
    """--dataset (reference image_train.py:19, read nowhere there): the named preset sets the image
    shape the command line left at its default, never an explicit flag; unknown names are labels."""
    fl = F.parse_flags(["--dataset=mnist"])
    assert F.apply_dataset_preset(fl) == {"output_size": 28, "c_dim": 1}
    assert (fl.output_size, fl.c_dim) == (28, 1)
    fl = F.parse_flags(["--dataset=mnist", "--output_size=32"])
    assert F.apply_dataset_preset(fl) == {"c_dim": 1} and fl.output_size == 32
    fl = F.parse_flags([])  # celebA: the reference shape, nothing to change
    assert F.apply_dataset_preset(fl) == {} and (fl.output_size, fl.c_dim) == (64, 3)
    fl = F.parse_flags(["--dataset=my_faces"])
    assert F.apply_dataset_preset(fl) == {}
    # data/<dataset> (carpedm20 layout) when --data_dir is left at a missing default
    monkeypatch.chdir(tmp_path)
    (tmp_path / "data" / "lsun").mkdir(parents=True)
    fl = F.parse_flags(["--dataset=lsun"])
    assert F.apply_dataset_preset(fl) == {"data_dir": "data/lsun"} and fl.data_dir == "data/lsun"


def test_log_device_placement_report(tmp_path, capsys):
    """--log_device_placement (reference image_train.py:36, default True, never used there): each
    rank prints where its work runs; --nolog_device_placement silences it."""
    from distributed_tensorflow_for_dcgan_amd.train import trainer
    base = ["--synthetic", "--max_steps=1", "--batch_size=4", "--output_size=28", "--c_dim=1", "--engine=reference",
            "--device=cpu", "--checkpoint_dir=%s" % (tmp_path / "ck"), "--sample_dir=%s" % (tmp_path / "s"),
            "--nosummaries", "--sample_every=0"]
    assert trainer.run(F.parse_flags(base)) == 0
    out = capsys.readouterr().out
    assert "[placement] /job:worker/replica:0/task:0/device:CPU:0" in out and "[placement] process group" in out
    assert trainer.run(F.parse_flags(base + ["--nolog_device_placement"])) == 0
    assert "[placement]" not in capsys.readouterr().out
