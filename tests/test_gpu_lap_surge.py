"""GPU: OCSORT-family first rounds with more detections than trackers (a crowd entering the scene).

association.py:20-28 pads such a problem with zero-cost dummy columns; which detections stay on
them sets the order of the unmatched list (association.py:179-199) and so the birth ids.  The
engines solve the transposed problem (trackers as rows, every one matched) and keep it only when
its optimum is certified unique (ocsort_common.hpp unique_optimum_tr); exact ties (e.g. a tracker
without velocity and without overlap has a row of exact zeros under plain IoU) fall back to the
lapjv replay.  Bar: every frame bit-exact against the oracle (which restates lapx's tie-breaking),
and the solver counters say which path ran.
"""
import time

import numpy as np
import pytest

from oracle.ocsort import OCSortOracle
from yolo_tracking_amd.synth import make_frames
from yolo_tracking_amd.trackers.ocsort import OCSortEngine

pytestmark = pytest.mark.gpu


def surge(n1, n2, nf, seed, start=2, canvas=None, **kw):
    """Population 1 on every frame; from frame `start` on population 2 (same canvas) appended."""
    a = make_frames(n1, nf, seed, canvas=canvas, **kw)
    b = make_frames(n2, nf, seed + 1000, canvas=canvas, **kw)
    return [a[f][0] if f < start else np.concatenate([a[f][0], b[f][0]]) for f in range(nf)]


@pytest.mark.parametrize("asso", ["giou", "iou", "diou"])
def test_ocsort_surge_matches_oracle(asso):
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, asso_threshold=0.3, delta_t=3,
              asso_func=asso, inertia=0.2, use_byte=False)
    frames = surge(300, 700, 8, 91, canvas=1600.0, low_conf_frac=0.0, drop_frac=0.05)
    shape = (1600, 1600, 3)
    eng = OCSortEngine(1, **kw)
    o = OCSortOracle(**kw)
    for f, d in enumerate(frames):
        got = eng.update([d], [shape])[0]
        exp = np.asarray(o.update(d, shape), dtype=np.float64).reshape(-1, 8)
        assert np.array_equal(got, exp), (asso, f)
    st = eng.state(0)
    assert np.array_equal(st["x"], np.array([k.kf.x.ravel() for k in o.trackers]).reshape(-1, 7))
    ls = eng.lap_stats()
    print(asso, ls)
    assert ls["transposed"] >= 1, ls
    assert ls["uncertified"] <= ls["transposed"]


def test_ocsort_multistream_surge_mixed_paths():
    """Four streams in one engine, two of them surging: the transposed solve, certified or not,
    runs per stream beside the normal orientation of the others."""
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, asso_threshold=0.3, delta_t=3,
              asso_func="iou", inertia=0.2, use_byte=False)
    streams = [surge(200, 300, 7, 120 + s, canvas=1200.0, low_conf_frac=0.0, drop_frac=0.05)
               if s % 2 == 0 else
               [d for d, _ in make_frames(200, 7, 120 + s, canvas=1200.0, low_conf_frac=0.0,
                                          drop_frac=0.05)]
               for s in range(4)]
    shape = (1200, 1200, 3)
    eng = OCSortEngine(4, **kw)
    ors = [OCSortOracle(**kw) for _ in range(4)]
    for f in range(7):
        got = eng.update([st[f] for st in streams], [shape] * 4)
        for s in range(4):
            exp = np.asarray(ors[s].update(streams[s][f], shape), dtype=np.float64).reshape(-1, 8)
            assert np.array_equal(got[s], exp), (s, f)


def test_deepocsort_2048_surge_solver_path():
    """The full-size DeepOCSORT surge golden (2048 trackers meet ~3900 detections): the transposed
    solve runs on the surge frames; bit-exact against the oracle; the frame time is printed."""
    import full_configs as fc
    from oracle.deepocsort import DeepOCSortOracle
    from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine
    g = fc.load()
    frames, img_shape, kw, warp, D = fc.deepocsort_frames(g, "dos_n2048_surge")
    eng = DeepOCSortEngine(1, feat_dim=D, **kw)
    o = DeepOCSortOracle(**kw)
    times = []
    for f, (d, feats) in enumerate(frames):
        t0 = time.perf_counter()
        out = eng.update([d], [feats], img_shapes=[img_shape])[0]
        times.append(time.perf_counter() - t0)
        ref = np.asarray(o.update(d, img_shape, feats, None), dtype=np.float64).reshape(-1, 8)
        assert np.array_equal(out, ref), f
    ls = eng.lap_stats()
    print("deepocsort surge", ls, "frame ms", [round(1e3 * t, 2) for t in times])
    assert ls["transposed"] >= 1, ls


def test_hybridsort_surge_matches_oracle():
    from oracle.hybridsort import HybridSortOracle
    from yolo_tracking_amd.trackers.hybridsort import HybridSortEngine
    HS_KW = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
                 asso_func="giou", inertia=0.2)
    D = 32
    a = make_frames(150, 7, 333, emb_dim=D, low_conf_frac=0.0, drop_frac=0.05)
    b = make_frames(250, 7, 1333, emb_dim=D, low_conf_frac=0.0, drop_frac=0.05)
    frames = [a[f] if f < 2 else (np.concatenate([a[f][0], b[f][0]]),
                                  np.concatenate([a[f][1], b[f][1]])) for f in range(7)]
    eng = HybridSortEngine(1, feat_dim=D, **HS_KW)
    o = HybridSortOracle(**HS_KW)
    nid = np.zeros(1, dtype=np.int64)
    for f, (d, e) in enumerate(frames):
        feats = e / np.linalg.norm(e)
        got = eng.update([d], [feats], next_id=nid)[0]
        exp = np.asarray(o.update(d, feats), dtype=np.float64).reshape(-1, 8)
        assert np.array_equal(got, exp), f
    print("hybridsort surge", eng.lap_stats())


# ------------------------------------------------------------------ the solve itself (KAT)
def _surge_like(rng, n_det, n_trk):
    """-(iou + angle) with more detections than trackers: each tracker has a strong pair, the
    rest of its column a small dense angle term (continuous: no exact ties)."""
    c = -0.1 * rng.random((n_det, n_trk))
    perm = rng.permutation(n_det)[:n_trk]
    for j in range(n_trk):
        if rng.random() < 0.95:
            c[perm[j], j] -= 0.3 + 0.7 * rng.random()
    return c


@pytest.mark.parametrize("na,nb", [(2, 1), (9, 4), (300, 100), (1000, 300), (3900, 2048),
                                   (5000, 700)])
@pytest.mark.parametrize("kind", ["uniform", "surge"])
def test_first_round_transposed_unique_matches_lapjv(na, nb, kind):
    """Tie-free costs, more rows than columns: the transposed solve is certified and equals
    lapjv's padded solution row for row."""
    from oracle.lap import lapjv
    from yolo_tracking_amd import _lib
    rng = np.random.default_rng(na * 31 + nb)
    c = rng.random((na, nb)) - 0.5 if kind == "uniform" else _surge_like(rng, na, nb)
    _, xo, _ = lapjv(c, extend_cost=True)
    rx, done, n_tight = _lib.lap_first_round(c)
    print(na, nb, kind, "tight edges", n_tight)
    assert done, n_tight
    assert np.array_equal(rx, xo), np.nonzero(rx != xo)[0][:10]


def test_first_round_transposed_ties_replay():
    """A column of exact zeros (a tracker without velocity or overlap, under IoU) ties every
    detection: not certified, so the engine replays lapjv."""
    from yolo_tracking_amd import _lib
    rng = np.random.default_rng(5)
    c = _surge_like(rng, 400, 150)
    c[:, 7] = 0.0
    c[:, 90] = 0.0
    _, done, n_tight = _lib.lap_first_round(c)
    assert not done, n_tight


def test_first_round_normal_orientation_unchanged():
    from oracle.lap import lapjv
    from yolo_tracking_amd import _lib
    rng = np.random.default_rng(8)
    c = rng.random((300, 500)) - 0.5
    _, xo, _ = lapjv(c, extend_cost=True)
    rx, done, n_tight = _lib.lap_first_round(c)
    assert done and n_tight == -1
    assert np.array_equal(rx, xo)


def _contested(rng, na, nb):
    """Random costs whose row minima crowd onto a tenth of the columns: many rows claim the same
    column, so the first-round solve's bidding rounds (lap_rect.hpp rect_arr) do real work."""
    c = rng.random((na, nb))
    hot = rng.integers(0, max(1, nb // 10), na)
    c[np.arange(na), hot] -= rng.random(na)
    return c


@pytest.mark.parametrize("na,nb,kind", [(1, 1, "uniform"), (5, 9, "contested"),
                                        (64, 64, "contested"), (300, 500, "contested"),
                                        (1000, 1000, "contested"), (2048, 2100, "contested"),
                                        (4096, 4264, "contested"), (4096, 4264, "uniform")])
def test_first_round_bidding_matches_lapjv(na, nb, kind):
    """Normal orientation (trackers >= detections), tie-free costs: the bidding rounds + searches
    return lapjv's assignment row for row (the optimum is unique), at the C4 / C5 sizes too (the
    rounds' duals in LDS up to the C5 shape)."""
    from oracle.lap import lapjv
    from yolo_tracking_amd import _lib
    rng = np.random.default_rng(na * 7 + nb)
    c = _contested(rng, na, nb) if kind == "contested" else rng.random((na, nb)) - 0.5
    _, xo, _ = lapjv(c, extend_cost=True)
    rx, done, n_tight = _lib.lap_first_round(c)
    assert done and n_tight == -1
    assert np.array_equal(rx, xo), np.nonzero(rx != xo)[0][:10]


@pytest.mark.parametrize("gap", [1e-10, 1e-9, 3e-9, 1e-8])
@pytest.mark.parametrize("scale", [1.0, 50.0])
def test_first_round_near_ties_uncertified_or_lapjv(gap, scale):
    """Near-tied alternative optima (an unmatched detection row given a matched pair's cost plus a
    reduced-cost gap of 1e-10 .. 1e-8, at unit scale and at 50x, as embedding- or long-term-
    weighted costs can be): the transposed solve is either left uncertified (the engine replays
    lapjv) or equals lapjv's solution row for row (the tolerance scales with the costs)."""
    from oracle.lap import lapjv
    from yolo_tracking_amd import _lib
    rng = np.random.default_rng(int(gap * 1e12) + int(scale))
    c = _surge_like(rng, 600, 200) * scale
    _, xo, _ = lapjv(c, extend_cost=True)
    free = np.nonzero(xo < 0)[0]
    used = np.nonzero(xo >= 0)[0]
    for k in range(8):   # eight near-tied swaps
        r, r2 = free[k], used[rng.integers(len(used))]
        c[r, xo[r2]] = c[r2, xo[r2]] + gap * scale
    _, xo, _ = lapjv(c, extend_cost=True)
    rx, done, n_tight = _lib.lap_first_round(c)
    print(gap, scale, "done", done, "tight", n_tight)
    assert (not done) or np.array_equal(rx, xo), np.nonzero(rx != xo)[0][:10]
