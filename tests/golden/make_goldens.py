#!/usr/bin/env python3
"""Generate golden vectors from the reference (container-only; needs /root/reference).

    python tests/golden/make_goldens.py            # writes tests/golden/*.npz

Fixtures (data only — inputs and the reference's outputs):
  G1 bytetrack_mot17.npz   ByteTrack on every MOT17-mini sequence (det.txt -> per-frame dets),
                           BaseTrack._count reset per sequence.
  G2 bytetrack_synth.npz   ByteTrack on seeded synthetic streams (yolo_tracking_amd.synth),
                           with the final Kalman state of every live track.
  G3 kat_*.npz             known-answer vectors: IoU family, fuse_score, ByteTrack KF
                           initiate / multi_predict / update, lapjv with and without cost_limit.
Every LAP call made while generating is tie-checked: the problem is re-solved on the row- and
column-reversed matrix and the matched real pairs must be identical; otherwise the fixture is
rejected (lapx's own tie-breaking is unpinned because lapx is not installed).
"""
import glob
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refshim  # noqa: E402
from yolo_tracking_amd.synth import make_frames  # noqa: E402

REF = refshim.REF
ref = refshim.load()

# ------------------------------------------------------------------ tie checking around lap.lapjv
_lap = sys.modules["lap"]
_orig_lapjv = _lap.lapjv
TIES = {"calls": 0, "ties": 0}


def _checked_lapjv(cost, extend_cost=False, cost_limit=np.inf, return_cost=True):
    opt, x, y = _orig_lapjv(cost, extend_cost=extend_cost, cost_limit=cost_limit)
    c = np.asarray(cost, dtype=np.double)
    if c.size:
        _, xf, _ = _orig_lapjv(c[::-1, ::-1], extend_cost=extend_cost, cost_limit=cost_limit)
        nr, nc = c.shape
        xf = xf[::-1]
        xf = np.where(xf >= 0, nc - 1 - xf, -1)
        TIES["calls"] += 1
        if not np.array_equal(np.asarray(x), xf):
            TIES["ties"] += 1
    return (opt, x, y) if return_cost else (x, y)


_lap.lapjv = _checked_lapjv


def run_bytetrack(frames, **kw):
    ref.basetrack.BaseTrack._count = 0
    t = ref.byte_tracker.BYTETracker(**kw)
    outs = []
    for dets in frames:
        o = t.update(dets, None)
        outs.append(np.asarray(o, dtype=np.float64).reshape(-1, 8))
    return t, outs


def pack_outputs(outs):
    counts = np.array([len(o) for o in outs], dtype=np.int32)
    rows = np.concatenate(outs, axis=0) if counts.sum() else np.zeros((0, 8))
    return counts, rows


def track_state(t):
    """Snapshot of every track in tracked_stracks then lost_stracks (list order)."""
    recs = []
    for lst, tag in ((t.tracked_stracks, 0), (t.lost_stracks, 1)):
        for s in lst:
            recs.append((tag, s.track_id, s.state, int(s.is_activated), s.frame_id, s.start_frame,
                         s.tracklet_len, s.mean, s.covariance))
    if not recs:
        return {}
    return dict(
        st_list=np.array([r[0] for r in recs], np.int32),
        st_id=np.array([r[1] for r in recs], np.int64),
        st_state=np.array([r[2] for r in recs], np.int32),
        st_act=np.array([r[3] for r in recs], np.int32),
        st_frame=np.array([r[4] for r in recs], np.int32),
        st_start=np.array([r[5] for r in recs], np.int32),
        st_len=np.array([r[6] for r in recs], np.int32),
        st_mean=np.stack([r[7] for r in recs]).astype(np.float64),
        st_cov=np.stack([r[8] for r in recs]).astype(np.float64),
    )


# ------------------------------------------------------------------ G1: MOT17-mini
def load_mot_dets(seq_dir):
    raw = np.loadtxt(os.path.join(seq_dir, "det", "det.txt"), delimiter=",")
    frames_idx = raw[:, 0].astype(int)
    n_frames = int(frames_idx.max())
    frames = []
    for f in range(1, n_frames + 1):
        r = raw[frames_idx == f]
        d = np.zeros((len(r), 6))
        d[:, 0] = r[:, 2]
        d[:, 1] = r[:, 3]
        d[:, 2] = r[:, 2] + r[:, 4]
        d[:, 3] = r[:, 3] + r[:, 5]
        d[:, 4] = r[:, 6]
        frames.append(d)
    return raw, frames


def make_g1():
    out = {}
    seqs = sorted(glob.glob(os.path.join(REF, "assets", "MOT17-mini", "train", "*")))
    names = []
    for sd in seqs:
        name = os.path.basename(sd)
        raw, frames = load_mot_dets(sd)
        before = dict(TIES)
        _, outs = run_bytetrack(frames, track_thresh=0.5, match_thresh=0.8, track_buffer=30,
                                frame_rate=30)
        counts, rows = pack_outputs(outs)
        # det.txt values carry <= 3 decimals: store them exactly as integers x 1000
        q = np.round(raw[:, [0, 2, 3, 4, 5, 6]] * 1000).astype(np.int64)
        assert np.array_equal(q / 1000.0, raw[:, [0, 2, 3, 4, 5, 6]]), name
        key = name.replace("-", "_")
        out[f"{key}__det_milli"] = q
        out[f"{key}__out_counts"] = counts
        out[f"{key}__out_box"] = rows[:, :4].astype(np.float64)
        out[f"{key}__out_int"] = rows[:, [4, 6, 7]].astype(np.int64)   # id, cls, det_ind
        out[f"{key}__out_score"] = rows[:, 5].astype(np.float64)
        names.append(name)
        print(f"G1 {name}: frames={len(frames)} dets={len(raw)} out_rows={len(rows)} "
              f"lap_calls={TIES['calls'] - before['calls']} ties={TIES['ties'] - before['ties']}")
    out["sequences"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "bytetrack_mot17.npz"), **out)


# ------------------------------------------------------------------ G2: synthetic streams
SYNTH_CASES = [  # (name, n_objects, n_frames, seed)
    ("n64_s11", 64, 40, 11),
    ("n256_s12", 256, 30, 12),
    ("n1024_s13", 1024, 6, 13),
]


def make_g2():
    out = {}
    for name, n, nf, seed in SYNTH_CASES:
        frames = [d for d, _ in make_frames(n, nf, seed)]
        before = dict(TIES)
        t, outs = run_bytetrack(frames, track_thresh=0.5, match_thresh=0.8, track_buffer=30,
                                frame_rate=30)
        ties = TIES["ties"] - before["ties"]
        assert ties == 0, f"{name}: {ties} tied LAP calls, choose another seed"
        counts, rows = pack_outputs(outs)
        out[f"{name}__dets"] = np.concatenate(frames, axis=0)
        out[f"{name}__det_counts"] = np.array([len(d) for d in frames], np.int32)
        out[f"{name}__out_counts"] = counts
        out[f"{name}__out"] = rows
        for k, v in track_state(t).items():
            out[f"{name}__{k}"] = v
        print(f"G2 {name}: out_rows={len(rows)} live_tracks={len(t.tracked_stracks)}+"
              f"{len(t.lost_stracks)} lap_calls={TIES['calls'] - before['calls']}")
    out["cases"] = np.array([c[0] for c in SYNTH_CASES])
    np.savez_compressed(os.path.join(HERE, "bytetrack_synth.npz"), **out)


# ------------------------------------------------------------------ G3: known-answer vectors
def rand_boxes(rng, n, canvas=200.0):
    xy = rng.uniform(0, canvas, size=(n, 2))
    wh = rng.uniform(2, 60, size=(n, 2))
    return np.concatenate([xy, xy + wh], axis=1)


def make_g3():
    rng = np.random.default_rng(2024)
    a = rand_boxes(rng, 37)
    b = rand_boxes(rng, 53)
    b[:5] = a[:5] + rng.normal(0, 2, size=(5, 4))  # guaranteed overlaps
    iou = ref.iou
    kat = dict(a=a, b=b,
               iou=iou.iou_batch(a, b), giou=iou.giou_batch(a, b), diou=iou.diou_batch(a, b),
               ciou=iou.ciou_batch(a, b), centroid=iou.centroid_batch(a, b, 640, 480))
    # fuse_score / iou_distance through the reference's STrack-free ndarray path
    scores = rng.uniform(0.1, 1.0, size=53)

    class _D:
        def __init__(self, s):
            self.score = s
    dist = ref.matching.iou_distance(list(a), list(b))
    kat["iou_distance"] = dist
    kat["det_scores"] = scores
    kat["fuse_score"] = ref.matching.fuse_score(dist.copy(), [_D(s) for s in scores])
    np.savez_compressed(os.path.join(HERE, "kat_iou.npz"), **kat)

    # ByteTrack KF (bytetrack_kf.py:55-226)
    kf = ref.bytetrack_kf.KalmanFilter()
    meas = np.concatenate([rng.uniform(50, 900, size=(40, 2)), rng.uniform(0.3, 1.2, size=(40, 1)),
                           rng.uniform(20, 200, size=(40, 1))], axis=1)
    init_m, init_c = zip(*[kf.initiate(z) for z in meas])
    init_m = np.stack(init_m)
    init_c = np.stack(init_c)
    m = init_m.copy()
    m[:, 4:] = rng.normal(0, 2, size=(40, 4))
    m[::3, 7] = 0
    c = init_c.copy()
    pm, pc = kf.multi_predict(m.copy(), c.copy())
    z = meas + rng.normal(0, 3, size=meas.shape)
    z[:, 2] = meas[:, 2] + rng.normal(0, 0.02, size=40)
    um, uc = zip(*[kf.update(pm[i], pc[i], z[i]) for i in range(40)])
    np.savez_compressed(os.path.join(HERE, "kat_kf_xyah.npz"), meas=meas, init_mean=init_m,
                        init_cov=init_c, pred_in_mean=m, pred_in_cov=c, pred_mean=pm, pred_cov=pc,
                        z=z, upd_mean=np.stack(um), upd_cov=np.stack(uc))

    # lapjv: cost_limit (matching.py:64) and padded (association.py:23), incl. rectangular/empty
    lap_cases = {}
    k = 0
    for (nr, nc, lim) in [(8, 8, 0.8), (12, 7, 0.5), (5, 19, 0.7), (30, 30, 0.8), (1, 1, 0.3),
                          (40, 25, np.inf), (9, 16, np.inf), (20, 20, np.inf), (0, 5, 0.8),
                          (6, 0, 0.8)]:
        cost = rng.random((nr, nc))
        ext = True
        before = TIES["ties"]
        opt, x, y = sys.modules["lap"].lapjv(cost, extend_cost=ext, cost_limit=lim)
        assert TIES["ties"] == before, "tied LAP KAT"
        lap_cases[f"c{k}__cost"] = cost
        lap_cases[f"c{k}__limit"] = np.array(lim)
        lap_cases[f"c{k}__x"] = np.asarray(x, np.int32)
        lap_cases[f"c{k}__y"] = np.asarray(y, np.int32)
        lap_cases[f"c{k}__opt"] = np.array(opt)
        k += 1
    lap_cases["n_cases"] = np.array(k)
    np.savez_compressed(os.path.join(HERE, "kat_lap.npz"), **lap_cases)
    print("G3 written")


if __name__ == "__main__":
    which = sys.argv[1:] or ["g1", "g2", "g3"]
    if "g3" in which:
        make_g3()
    if "g1" in which:
        make_g1()
    if "g2" in which:
        make_g2()
    print(f"LAP calls {TIES['calls']}, tied {TIES['ties']}")
