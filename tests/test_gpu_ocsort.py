"""GPU: the device-resident OCSORT engine against the reference goldens (G5) and the oracle.

Bar: outputs equal to the reference's up to the numbering of same-frame births on every case, and
bit-exact (ids, output order, boxes, Kalman state) wherever the oracle is (G5 `exact` flag: lapx
near-ties among discarded pairs decide birth order, see make_goldens.py); the engine against the
oracle frame by frame; the Kalman filter (incl. freeze / virtual-trajectory replay) bit-exact.
"""
import os

import numpy as np
import pytest

from oracle.ocsort import KF7, OCSortOracle, bbox_to_z
from test_oracle_golden import OCSORT_CASES, canonical_equal, golden_outputs, ocsort_case
from yolo_tracking_amd import _lib, create_tracker, get_tracker_config
from yolo_tracking_amd.synth import make_frames
from yolo_tracking_amd.trackers.ocsort import KalmanBoxTracker, OCSortEngine

pytestmark = pytest.mark.gpu


def test_kf7_sequences_match_oracle():
    rng = np.random.default_rng(3)
    n, steps = 300, 30
    boxes = np.cumsum(rng.normal(0, 3, size=(steps + 1, n, 4)), axis=0)
    base = np.column_stack([rng.uniform(50, 900, n), rng.uniform(50, 900, n),
                            rng.uniform(60, 120, n), rng.uniform(60, 120, n)])
    xyxy = np.empty_like(boxes)
    for s in range(steps + 1):
        c = base[:, :2] + boxes[s, :, :2]
        wh = np.abs(base[:, 2:] + boxes[s, :, 2:]) + 5
        xyxy[s] = np.column_stack([c - wh / 2, c + wh / 2])
    z = np.array([[bbox_to_z(xyxy[s, i]).ravel() for i in range(n)] for s in range(steps + 1)])
    miss = rng.random((steps, n)) < 0.3
    miss[:, ::7] = False
    zz = z[1:].copy()
    zz[miss] = np.nan
    x, P = _lib.kf7_run(z[0], zz)
    for i in range(n):
        kf = KF7(z[0, i].reshape(4, 1))
        for s in range(steps):
            kf.predict()
            kf.update(None if miss[s, i] else zz[s, i].reshape(4, 1))
        assert np.array_equal(x[i], kf.x.ravel()), i
        assert np.array_equal(P[i], kf.P), i


def _run_engine(frames, img_shape, kw):
    eng = OCSortEngine(1, **kw)
    outs = [eng.update([d], [img_shape])[0] for d in frames]
    return eng, outs


@pytest.mark.parametrize("name", OCSORT_CASES)
def test_ocsort_golden(golden_dir, name):
    g = np.load(os.path.join(golden_dir, "ocsort_synth.npz"))
    frames, img_shape, kw = ocsort_case(g, name)
    eng, got = _run_engine(frames, img_shape, kw)
    exp = golden_outputs(g, name)
    assert canonical_equal(got, exp)
    # the oracle, frame by frame (same solver sequence, same costs)
    o = OCSortOracle(**kw)
    for f, d in enumerate(frames):
        ref = np.asarray(o.update(d, img_shape), dtype=np.float64).reshape(-1, 8)
        assert np.array_equal(got[f], ref), (name, f)
    st = eng.state(0)
    assert np.array_equal(st["x"], np.array([k.kf.x.ravel() for k in o.trackers]).reshape(-1, 7))
    assert np.array_equal(st["P"], np.array([k.kf.P for k in o.trackers]).reshape(-1, 7, 7))
    if bool(g[f"{name}__exact"]):
        assert all(np.array_equal(a, b) for a, b in zip(got, exp))
        assert np.array_equal(st["id"], g[f"{name}__st_id"])
        assert np.array_equal(st["x"], g[f"{name}__st_x"])
        assert np.array_equal(st["P"], g[f"{name}__st_P"])
        ints = np.column_stack([st["age"], st["hits"], st["hit_streak"], st["time_since_update"],
                                st["observed"], st["saved"]])
        assert np.array_equal(ints, g[f"{name}__st_int"])


def test_ocsort_python_surface(golden_dir):
    g = np.load(os.path.join(golden_dir, "ocsort_synth.npz"))
    name = "oc_n64_dt5"
    frames, img_shape, kw = ocsort_case(g, name)
    img = np.zeros((img_shape[0], img_shape[1], 3), np.uint8)
    from yolo_tracking_amd.trackers.ocsort import OCSort
    t = OCSort(per_class=False, **kw)
    exp = golden_outputs(g, name)
    for f, d in enumerate(frames):
        got = np.asarray(t.update(d, img)).reshape(-1, 8)
        assert np.array_equal(got, exp[f]), f
    # create_tracker reads ocsort.yaml; empty frames return np.array([])
    tz = create_tracker("ocsort", get_tracker_config("ocsort"), None, "0", False, False)
    assert KalmanBoxTracker.count == 0
    r = tz.update(frames[0], img)
    assert r.shape == (len(frames[0]), 8)   # frame_count <= min_hits: frame 1's births reported
    assert KalmanBoxTracker.count == len(frames[0])
    r = tz.update(np.empty((0, 6)), img)
    assert r.shape == (0,)


def test_ocsort_multistream_matches_oracle():
    S, n, nf = 4, 96, 15
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, asso_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2, use_byte=False)
    streams = [[d for d, _ in make_frames(n, nf, 200 + s, low_conf_frac=0.0, drop_frac=0.1)]
               for s in range(S)]
    eng = OCSortEngine(S, **kw, track_capacity=64, max_dets=32)   # grows on demand
    ors = [OCSortOracle(**kw) for _ in range(S)]
    shape = (640, 640, 3)
    for f in range(nf):
        got = eng.update([streams[s][f] for s in range(S)], [shape] * S)
        for s in range(S):
            exp = np.asarray(ors[s].update(streams[s][f], shape), dtype=np.float64).reshape(-1, 8)
            assert np.array_equal(got[s], exp), (s, f)
