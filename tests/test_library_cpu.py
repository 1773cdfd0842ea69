"""CPU: the HIP library and the package load; every C-ABI symbol declared in include/*.h is
exported; the plugin surface mirrors the reference's.  No compute calls (no GPU here)."""
import glob
import os
import re

import numpy as np
import pytest

from conftest import REPO


def _declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        names |= set(re.findall(r"^\s*(?:int|const char \*)\s*(yta_\w+)\s*\(", src, re.M))
    return names


def test_library_exports_every_declared_symbol():
    from yolo_tracking_amd import _lib
    lib = _lib.load_library()
    declared = _declared_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(_lib.EXPORTED_SYMBOLS) == declared
    assert lib.yta_version() >= 1


def test_missing_library_fails_loudly(tmp_path):
    from yolo_tracking_amd import _lib
    with pytest.raises(_lib.YTAError):
        _lib.load_library(str(tmp_path / "nope.so"))


def test_plugin_surface():
    import yolo_tracking_amd as y
    assert y.TRACKERS == ['bytetrack', 'botsort', 'strongsort', 'ocsort', 'deepocsort',
                          'hybridsort']
    for t in y.TRACKERS:
        assert y.get_tracker_config(t).exists(), t
    import yaml
    cfg = yaml.safe_load(open(y.get_tracker_config("bytetrack")))
    assert cfg["track_thresh"] == 0.5 and cfg["match_thresh"] == 0.8
    assert cfg["track_buffer"] == 30 and cfg["frame_rate"] == 30


def test_unknown_tracker_exits():
    import yolo_tracking_amd as y
    with pytest.raises(SystemExit):
        y.create_tracker("nope", y.get_tracker_config("bytetrack"), None, "cpu", False, False)


def test_device_parsing():
    from yolo_tracking_amd._lib import parse_device
    assert parse_device("cpu") == 0 and parse_device("0") == 0 and parse_device("cuda:3") == 3
    assert parse_device(2) == 2 and parse_device(None) == 0 and parse_device("1,2") == 1


def test_synthetic_stream_is_deterministic():
    from yolo_tracking_amd.synth import make_frames
    a = make_frames(128, 3, seed=5)
    b = make_frames(128, 3, seed=5)
    for (da, _), (db, _) in zip(a, b):
        assert np.array_equal(da, db)
    assert a[0][0].shape == (128, 6)


def test_default_cmc_is_sparse_opt_flow():
    """Without cmc= the trackers get SparseOptFlow, as in the reference (bot_sort.py:228,
    deep_ocsort.py:351); constructing it touches no GPU (the engine starts with the first frame)."""
    from yolo_tracking_amd.motion import (ECC, IdentityCMC, SparseOptFlow, default_cmc,
                                          get_cmc_method)
    assert isinstance(default_cmc("BoTSORT"), SparseOptFlow)
    assert get_cmc_method("sof") is SparseOptFlow
    assert get_cmc_method("ecc") is ECC and isinstance(ECC(), ECC)
    with pytest.raises(NotImplementedError):
        get_cmc_method("orb")
    assert np.array_equal(IdentityCMC().apply(None, None), np.eye(2, 3))
