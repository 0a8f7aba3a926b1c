"""CPU tests of the tile-table tooling: the in-situ tuner only proposes legal neighbours, and the
shipped table's entries name configurations the kernels accept (LDS ring within 160 KiB, known
tile ids / stage counts)."""
import json
import os

import pytest

from distributed_tensorflow_for_dcgan_amd.ops import hip as H


def test_tuner_neighbours_fit_lds():
    T = pytest.importorskip("benchmarks.tune_insitu")
    for key, cur in (("1,256,8,8,256,16,16,128", (216, 1)), ("0,128,32,32,64,16,16,128", (210, 1)),
                     ("1,512,4,4,2048,8,8,1024", (210, 2))):
        for tiles in (False, True):
            for cfg, sp in T.neighbours(key, cur, tiles=tiles):
                assert sp >= 1
                if 200 <= cfg < 300:
                    assert cfg % 10 in H.IGEMM3_TILES and H.igemm3_lds(cfg) <= 160 * 1024, (key, cfg)


def test_shipped_table_entries_are_legal():
    path = os.path.join(os.path.dirname(H.__file__), "igemm_tuned.json")
    with open(path) as f:
        table = json.load(f)
    assert table
    for key, val in table.items():
        cfg, sp = (int(x) for x in val.split(":"))
        assert sp >= 1, key
        if key.startswith("w3,") and cfg >= 400:
            f = key.split(",")
            assert H.wgrad5_fits(cfg, int(f[1]), int(f[4]), int(f[5]), int(f[3])), (key, val)
        elif key.startswith("w3,"):
            assert 300 <= cfg < 340 and cfg % 10 in H.WGRAD3_TILES, (key, val)
        elif cfg >= 200:
            assert cfg < 240 and cfg % 10 in H.IGEMM3_TILES and H.igemm3_lds(cfg) <= 160 * 1024, (key, val)
        else:
            assert cfg % 100 in H.IGEMM_CFGS and sp == 1, (key, val)


def test_tuner_offers_fitting_wgrad5_configs():
    """The in-situ tuner's weight-gradient neighbours include exactly the wgrad5 configurations
    whose channel count and output width match the layer."""
    T = pytest.importorskip("benchmarks.tune_insitu")
    nb = T.neighbours("w3,64,128,128,16,16,32", (311, 16))
    assert {(400, 16), (401, 16), (410, 16)} <= set(nb)
    assert not any(c in (402, 403, 404, 405, 406, 407) for c, _ in nb)
    nb = T.neighbours("w3,128,256,256,8,8,16", (310, 4))
    assert {(402, 4), (404, 4), (406, 4), (412, 4)} <= set(nb) and not any(c in (400, 401, 405) for c, _ in nb)
