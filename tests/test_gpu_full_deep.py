"""GPU: the BASELINE.json configs at their stated sizes, run long enough to reach the lifecycle
paths, against the reference's goldens (tests/golden/make_goldens_deep.py -> full_deep.npz).

  * C3 BoT-SORT 1024 x 1024, D 512, 65 frames with 5 % missed detections: Lost tracks re-found
    (bot_sort.py:339-346) and expired after max_time_lost = 60 (bot_sort.py:386-390).
  * C4 DeepOCSORT 2048 x 2048, D 512, CMC affine, 2 streams x 40 frames in one engine launch per
    frame: ORU re-acquisitions (deep_ocsort.py:220-232) and deaths after max_age = 30
    (deep_ocsort.py:514-517).
  * C5 HybridSORT 4096 x 4096, D 512: one stream x 35 frames (deaths after max_age,
    hybridsort.py:562-567; 30-deep feature banks, hybridsort.py:190, :438-439), and the config's
    per-GPU concurrency, 8 streams x 12 frames in one engine launch per frame.

Bar as tests/test_gpu_full_configs.py: every frame of every stream bit-exact (row count, SHA-256
of the reference's rows, the last frame in full); final states: ids exact, Kalman state bit-exact
(BoT-SORT, HybridSORT) or within 1e-9 (DeepOCSORT under the camera warp).
"""
import numpy as np
import pytest

import full_configs as fc
from test_oracle_golden import reid_features

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    return fc.load_deep()


def test_botsort_1024_d512_65_frames_expiry(g):
    from yolo_tracking_amd.trackers.botsort import BoTSORTEngine
    name = "bs_n1024_d512_f65"
    assert int(g[f"{name}__removed"]) > 0          # the reference expired tracks in this case
    frames, params, D = fc.botsort_frames(g, name)
    eng = BoTSORTEngine(1, feat_dim=D, **params)
    for f, (dets, embs) in enumerate(frames):
        feats = reid_features(dets, embs, params["track_high_thresh"])
        fc.check_frame(g, name, f, eng.update([dets], [feats])[0])
    st = eng.state(0)
    assert np.array_equal(st["list"], g[f"{name}__st_list"])
    assert np.array_equal(st["id"], g[f"{name}__st_id"])
    assert np.array_equal(st["mean"], g[f"{name}__st_mean"])
    assert np.array_equal(st["cov"][::64], g[f"{name}__st_cov_sample"])
    feats, _, _ = eng.features(0)
    np.testing.assert_allclose(feats[::64], g[f"{name}__st_feat_sample"], rtol=1e-5, atol=1e-6)


def test_deepocsort_2048_cmc_40_frames_two_streams(g):
    from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine
    cases = [fc.deepocsort_frames(g, n) for n in fc.DOS_F40]
    kw, D = cases[0][2], cases[0][4]
    assert all(c[2] == kw for c in cases)
    eng = DeepOCSortEngine(len(cases), feat_dim=D, **kw)
    warps = np.stack([c[3] for c in cases])
    nf = len(cases[0][0])
    assert nf > kw["max_age"] + 2
    for f in range(nf):
        outs = eng.update([c[0][f][0] for c in cases], [c[0][f][1] for c in cases], warps=warps,
                          img_shapes=[c[1] for c in cases])
        for s, name in enumerate(fc.DOS_F40):
            fc.check_frame(g, name, f, outs[s])
    for s, name in enumerate(fc.DOS_F40):
        st = eng.state(s)
        assert np.array_equal(st["id"], g[f"{name}__st_id"])
        np.testing.assert_allclose(st["x"], g[f"{name}__st_x"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(st["P"][::64], g[f"{name}__st_P_sample"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(st["emb"][::64], g[f"{name}__st_emb_sample"], rtol=0,
                                   atol=1e-12)


def _hybridsort_run(g, names):
    from yolo_tracking_amd.trackers.hybridsort import HybridSortEngine
    cases = [fc.hybridsort_frames(g, n) for n in names]
    kw, D = cases[0][1], cases[0][2]
    S = len(cases)
    eng = HybridSortEngine(S, feat_dim=D, **kw)
    nid = np.zeros(S, dtype=np.int64)
    for f in range(len(cases[0][0])):
        dets = [c[0][f][0] for c in cases]
        feats = [c[0][f][1] / np.linalg.norm(c[0][f][1]) for c in cases]
        outs = eng.update(dets, feats, next_id=nid)
        for s, name in enumerate(names):
            fc.check_frame(g, name, f, outs[s])
    for s, name in enumerate(names):
        st = eng.state(s)
        assert np.array_equal(st["id"], g[f"{name}__st_id"])
        assert np.array_equal(st["x"], g[f"{name}__st_x"])
        assert np.array_equal(st["P"][::64], g[f"{name}__st_P_sample"])
        np.testing.assert_allclose(st["feat"][::64], g[f"{name}__st_feat_sample"], rtol=0,
                                   atol=2e-7)
        assert nid[s] == int(g[f"{name}__count"])


def test_hybridsort_4096_35_frames_deaths(g):
    name = "hs_n4096_f35"
    assert int(g[f"{name}__gen"][1]) > 32
    _hybridsort_run(g, [name])


def test_hybridsort_4096_eight_streams_one_launch(g):
    _hybridsort_run(g, fc.HS_S8)


def test_ocsort_256_45_frames_deaths(g):
    """C2 OCSORT 256 x 256 (GIoU) past max_age = 30 with ORU re-acquisitions: every frame
    bit-exact, final Kalman states bit-exact, the ID counter."""
    from yolo_tracking_amd.trackers.ocsort import OCSortEngine
    name = "oc_n256_f45"
    n, nf, seed = (int(x) for x in g[f"{name}__gen"])
    low, drop = (float(x) for x in g[f"{name}__stream"])
    frames = [d for d, _ in fc.make_frames(n, nf, seed, low_conf_frac=low, drop_frac=drop)]
    assert float(np.sum([d.sum() for d in frames])) == g[f"{name}__in_sum"][0]
    p = g[f"{name}__params"]
    kw = dict(det_thresh=float(p[0]), max_age=int(p[1]), min_hits=int(p[2]),
              asso_threshold=float(p[3]), delta_t=int(p[4]), inertia=float(p[5]),
              use_byte=bool(p[6]), asso_func=str(g[f"{name}__asso"]))
    shape = tuple(int(v) for v in g[f"{name}__img"]) + (3,)
    eng = OCSortEngine(1, **kw)
    nid = np.zeros(1, np.int64)
    for f, d in enumerate(frames):
        fc.check_frame(g, name, f, eng.update([d], [shape], next_id=nid)[0])
    st = eng.state(0)
    assert np.array_equal(st["id"], g[f"{name}__st_id"])
    assert np.array_equal(st["x"], g[f"{name}__st_x"])
    assert np.array_equal(st["P"][::64], g[f"{name}__st_P_sample"])
    assert nid[0] == int(g[f"{name}__count"])


def test_botsort_1024_d512_cmc_warp_30_frames(g):
    """C3 BoT-SORT at size under the §8(d) CMC warp every frame (multi_gmc): ids, order,
    det_ind, scores and classes exact every frame, boxes and final states within 1e-9 relative
    (the warped covariance path is not the reference's operation order)."""
    from yolo_tracking_amd.trackers.botsort import BoTSORTEngine
    name = "bs_n1024_d512_cmc_f30"
    frames, params, D = fc.botsort_frames(g, name)
    warp = g[f"{name}__warp"]
    eng = BoTSORTEngine(1, feat_dim=D, **params)
    counts = g[f"{name}__out_counts"]
    offs = np.concatenate([[0], np.cumsum(counts)])
    rows = g[f"{name}__out"]
    for f, (dets, embs) in enumerate(frames):
        feats = reid_features(dets, embs, params["track_high_thresh"])
        out = eng.update([dets], [feats], warps=warp[None])[0]
        exp = rows[offs[f]:offs[f + 1]]
        assert out.shape == exp.shape, (f, out.shape, exp.shape)
        assert np.array_equal(out[:, 4:], exp[:, 4:]), f
        np.testing.assert_allclose(out[:, :4], exp[:, :4], rtol=1e-9, atol=1e-9, err_msg=str(f))
    st = eng.state(0)
    assert np.array_equal(st["list"], g[f"{name}__st_list"])
    assert np.array_equal(st["id"], g[f"{name}__st_id"])
    np.testing.assert_allclose(st["mean"], g[f"{name}__st_mean"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(st["cov"][::64], g[f"{name}__st_cov_sample"], rtol=1e-9,
                               atol=1e-9)
