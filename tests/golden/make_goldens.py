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
  G4 botsort_synth.npz     BoT-SORT (botsort.yaml parameters) on seeded synthetic streams with
                           embeddings (fake ReID = harness rows / global norm, fake CMC = harness
                           warp: identity or SURVEY §8(d)'s fixed affine), final Kalman states and
                           smoothed features.  Every embedding-threshold comparison and every LAP
                           cost is margin-checked (> 1e-6 from its threshold), so a tolerance-level
                           difference in float32 embedding arithmetic cannot flip an assignment.
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


# ------------------------------------------------------------------ G4: BoT-SORT
BOTSORT_YAML = dict(track_high_thresh=0.33824964456239337, track_low_thresh=0.1,
                    new_track_thresh=0.21144301345190655, track_buffer=60,
                    match_thresh=0.22734550911325851, proximity_thresh=0.5945380911899254,
                    appearance_thresh=0.4818211117541298, frame_rate=30)   # botsort.yaml
CMC_AFFINE = np.array([[1.0, 1e-3, 0.5], [-1e-3, 1.0, -0.3]])
BOTSORT_CASES = [  # (name, n_objects, n_frames, seed, emb_dim, warp, extra kwargs)
    ("bs_n64_d32", 64, 30, 41, 32, None, {}),
    ("bs_n256_d64", 256, 20, 42, 64, None, {}),
    ("bs_n256_d64_cmc", 256, 20, 43, 64, CMC_AFFINE, {}),
    ("bs_n128_fuse", 128, 25, 44, 32, None, {"fuse_first_associate": True}),
    ("bs_n128_noreid", 128, 25, 45, 0, None, {"with_reid": False}),
    ("bs_n512_d128", 512, 4, 46, 128, None, {}),
]
MARGIN = {"min": np.inf}


def _margin(vals, thr):
    v = np.asarray(vals, dtype=np.float64).ravel()
    v = v[np.isfinite(v)]
    if v.size:
        MARGIN["min"] = min(MARGIN["min"], float(np.min(np.abs(v - thr))))


def make_g4():
    bs = refshim.load_botsort()
    H = refshim.Harness
    mod = bs.bot_sort
    orig_emb = mod.embedding_distance

    CHECK_IOU = {"on": False}
    orig_iou = mod.iou_distance

    def emb_checked(tracks, dets, metric="cosine"):
        e = orig_emb(tracks, dets, metric)
        if e.size:   # only entries the proximity mask leaves in play can change a cost
            live = orig_iou(tracks, dets) <= BOTSORT_YAML["proximity_thresh"]
            h = (e / 2.0)[live]
            for thr in (BOTSORT_YAML["appearance_thresh"], BOTSORT_YAML["match_thresh"], 0.7):
                _margin(h, thr)
        return e

    def iou_checked(a, b):
        d = orig_iou(a, b)
        if CHECK_IOU["on"]:   # Kalman states under a non-identity warp are not bit-exact
            for thr in (0.5, 0.7, 0.15, BOTSORT_YAML["proximity_thresh"],
                        BOTSORT_YAML["match_thresh"]):
                _margin(d, thr)
        return d

    mod.embedding_distance, mod.iou_distance = emb_checked, iou_checked
    out = {}
    try:
        for name, n, nf, seed, D, warp, extra in BOTSORT_CASES:
            frames = make_frames(n, nf, seed, emb_dim=max(D, 1))
            before = dict(TIES)
            MARGIN["min"] = np.inf
            kw = dict(BOTSORT_YAML, **extra)
            t = mod.BoTSORT(None, "cpu", False, **kw)
            H.high_thresh = kw["track_high_thresh"]
            H.warp = np.eye(2, 3) if warp is None else warp
            CHECK_IOU["on"] = warp is not None
            outs = []
            img = np.zeros((8, 8, 3), np.uint8)
            for dets, embs in frames:
                H.dets, H.feats = dets, embs
                outs.append(np.asarray(t.update(dets, img), dtype=np.float64).reshape(-1, 8))
            ties = TIES["ties"] - before["ties"]
            assert ties == 0, f"{name}: {ties} tied LAP calls"
            assert MARGIN["min"] > 1e-6, f"{name}: threshold margin {MARGIN['min']}"
            counts, rows = pack_outputs(outs)
            # inputs are regenerated by the tests from (n, frames, seed, D) with
            # yolo_tracking_amd.synth; the checksums pin that generator
            out[f"{name}__gen"] = np.array([n, nf, seed, D], np.int64)
            out[f"{name}__in_sum"] = np.array(
                [float(np.sum([d.sum() for d, _ in frames])),
                 float(np.sum([e.astype(np.float64).sum() for _, e in frames])) if D else 0.0])
            out[f"{name}__warp"] = np.asarray(H.warp, dtype=np.float64)
            out[f"{name}__params"] = np.array([kw["track_high_thresh"], kw["track_low_thresh"],
                                               kw["new_track_thresh"], kw["track_buffer"],
                                               kw["match_thresh"], kw["proximity_thresh"],
                                               kw["appearance_thresh"], kw["frame_rate"],
                                               float(kw.get("fuse_first_associate", False)),
                                               float(kw.get("with_reid", True))])
            out[f"{name}__out_counts"] = counts
            out[f"{name}__out"] = rows
            recs = [(tag, s) for lst, tag in ((t.tracked_stracks, 0), (t.lost_stracks, 1))
                    for s in lst]
            out[f"{name}__st_list"] = np.array([r[0] for r in recs], np.int64)
            out[f"{name}__st_id"] = np.array([r[1].id for r in recs], np.int64)
            out[f"{name}__st_state"] = np.array([r[1].state for r in recs], np.int64)
            out[f"{name}__st_act"] = np.array([int(r[1].is_activated) for r in recs], np.int64)
            out[f"{name}__st_frame"] = np.array([r[1].frame_id for r in recs], np.int64)
            out[f"{name}__st_start"] = np.array([r[1].start_frame for r in recs], np.int64)
            out[f"{name}__st_len"] = np.array([r[1].tracklet_len for r in recs], np.int64)
            out[f"{name}__st_mean"] = np.array([r[1].mean for r in recs]).reshape(-1, 8)
            out[f"{name}__st_cov"] = np.array([r[1].covariance for r in recs]).reshape(-1, 8, 8)
            if D:
                out[f"{name}__st_feat"] = np.array([r[1].smooth_feat for r in recs],
                                                   np.float32).reshape(-1, D)
            print(f"G4 {name}: out_rows={len(rows)} live={len(t.tracked_stracks)}+"
                  f"{len(t.lost_stracks)} lap_calls={TIES['calls'] - before['calls']} "
                  f"min_margin={MARGIN['min']:.3g}")
    finally:
        mod.embedding_distance, mod.iou_distance = orig_emb, orig_iou
    out["cases"] = np.array([c[0] for c in BOTSORT_CASES])
    np.savez_compressed(os.path.join(HERE, "botsort_synth.npz"), **out)


# ------------------------------------------------------------------ G5: OCSORT
OCSORT_YAML = dict(det_thresh=0.0, max_age=30, min_hits=1, asso_threshold=0.3, delta_t=3,
                   asso_func="giou", inertia=0.2, use_byte=False)             # ocsort.yaml
OCSORT_CASES = [  # (name, n_objects, n_frames, seed, stream kwargs, tracker kwargs)
    ("oc_n64_giou", 64, 30, 51, dict(drop_frac=0.05), {}),
    ("oc_n256_giou", 256, 20, 52, dict(drop_frac=0.05), {}),
    ("oc_n128_iou_mh3", 128, 25, 53, dict(drop_frac=0.08),
     dict(asso_func="iou", min_hits=3, det_thresh=0.2, max_age=5)),
    ("oc_n128_diou", 128, 20, 54, dict(drop_frac=0.05), dict(asso_func="diou")),
    ("oc_n128_ciou", 128, 20, 55, dict(drop_frac=0.05), dict(asso_func="ciou")),
    ("oc_n96_centroid", 96, 15, 56, dict(drop_frac=0.05), dict(asso_func="centroid")),
    ("oc_n128_byte", 128, 20, 57, dict(drop_frac=0.05, low_conf_frac=0.2),
     dict(use_byte=True, det_thresh=0.5, asso_func="iou")),
    ("oc_n64_dt5", 64, 40, 58, dict(drop_frac=0.15), dict(delta_t=5, inertia=0.4)),
]


def canonical_equal(outs_a, outs_b):
    """Equal up to the numbering of tracks born in the same frame: per frame the rows are matched
    by det_ind (unique per output row) and must agree in box, conf, cls; ids must correspond
    through one bijection over the whole stream."""
    fwd, bwd = {}, {}
    for a, b in zip(outs_a, outs_b):
        if a.shape != b.shape:
            return False
        if not len(a):
            continue
        a = a[np.argsort(a[:, 7], kind="stable")]
        b = b[np.argsort(b[:, 7], kind="stable")]
        if not np.array_equal(a[:, [0, 1, 2, 3, 5, 6, 7]], b[:, [0, 1, 2, 3, 5, 6, 7]]):
            return False
        for ia, ib in zip(a[:, 4], b[:, 4]):
            if fwd.setdefault(ia, ib) != ib or bwd.setdefault(ib, ia) != ia:
                return False
    return True


def _oracle_lockstep(frames, img_shape, kw, outs):
    """The oracle (lapx restated in oracle/lapjv.c) must reproduce the reference outputs (SciPy
    stand-in for lapx) up to the numbering of same-frame births, also with every padded LAP solved
    on a perturbed (1e-9 relative noise), row/column-reversed cost matrix: no near-tie may decide
    which detections and tracks are matched.  Near-ties among the discarded pairs only permute the
    order of same-frame births (the unmatched lists, association.py:179-199).  Returns whether the
    oracle matched the reference exactly (birth order included)."""
    import oracle.ocsort as oc
    orig = oc.linear_assignment_padded
    rng = np.random.default_rng(7)

    def perturbed(cost):
        c = np.asarray(cost, np.float64)
        c = c * (1.0 + 1e-9 * rng.standard_normal(c.shape))
        m = orig(c[::-1, ::-1])
        if m.size == 0:
            return m
        m = np.stack([c.shape[0] - 1 - m[:, 0], c.shape[1] - 1 - m[:, 1]], axis=1)
        return m[np.argsort(m[:, 0])]

    exact = None
    for lap_fn in (orig, perturbed):
        oc.linear_assignment_padded = lap_fn
        try:
            t = oc.OCSortOracle(**kw)
            got = [np.asarray(t.update(d, img_shape), dtype=np.float64).reshape(-1, 8)
                   for d, _ in frames]
        finally:
            oc.linear_assignment_padded = orig
        assert canonical_equal(got, outs), lap_fn.__name__
        if exact is None:
            exact = all(np.array_equal(g, o) for g, o in zip(got, outs))
    return exact


def make_g5():
    mod = ref.ocsort
    out = {}
    for name, n, nf, seed, skw, tkw in OCSORT_CASES:
        skw = dict(skw)
        skw.setdefault("low_conf_frac", 0.0)
        frames = make_frames(n, nf, seed, **skw)
        from yolo_tracking_amd.synth import SyntheticStream
        img_shape = SyntheticStream(n, seed, **skw).img_shape
        kw = dict(OCSORT_YAML, **tkw)
        t = mod.OCSort(per_class=False, **kw)
        img = np.zeros((img_shape[0], img_shape[1], 3), np.uint8)
        outs = [np.asarray(t.update(d, img), dtype=np.float64).reshape(-1, 8) for d, _ in frames]
        exact = _oracle_lockstep(frames, img_shape, kw, outs)
        counts, rows = pack_outputs(outs)
        out[f"{name}__exact"] = np.array(exact)
        out[f"{name}__gen"] = np.array([n, nf, seed], np.int64)
        out[f"{name}__stream"] = np.array([skw["low_conf_frac"], skw.get("drop_frac", 0.0)])
        out[f"{name}__in_sum"] = np.array([float(np.sum([d.sum() for d, _ in frames]))])
        out[f"{name}__img"] = np.array(img_shape[:2], np.int64)
        out[f"{name}__params"] = np.array([kw["det_thresh"], kw["max_age"], kw["min_hits"],
                                           kw["asso_threshold"], kw["delta_t"], kw["inertia"],
                                           float(kw["use_byte"])])
        out[f"{name}__asso"] = np.array(kw["asso_func"])
        out[f"{name}__out_counts"] = counts
        out[f"{name}__out"] = rows
        trk = t.trackers
        out[f"{name}__st_id"] = np.array([k.id for k in trk], np.int64)
        out[f"{name}__st_x"] = np.array([k.kf.x.ravel() for k in trk]).reshape(-1, 7)
        out[f"{name}__st_P"] = np.array([k.kf.P for k in trk]).reshape(-1, 7, 7)
        out[f"{name}__st_int"] = np.array([[k.age, k.hits, k.hit_streak, k.time_since_update,
                                            int(k.kf.observed), int(k.kf.attr_saved is not None)]
                                           for k in trk], np.int64).reshape(-1, 6)
        print(f"G5 {name}: out_rows={len(rows)} live={len(trk)} oracle_exact={exact}")
    out["cases"] = np.array([c[0] for c in OCSORT_CASES])
    np.savez_compressed(os.path.join(HERE, "ocsort_synth.npz"), **out)


# ------------------------------------------------------------------ G6: DeepOCSORT
DEEPOCSORT_YAML = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
                       asso_func="giou", inertia=0.2, w_association_emb=0.75,
                       alpha_fixed_emb=0.95, aw_param=0.5, embedding_off=False, cmc_off=False,
                       aw_off=False)                                    # deepocsort.yaml
DEEPOCSORT_CASES = [  # (name, n_objects, n_frames, seed, emb_dim, warp, stream kw, tracker kw)
    ("dos_n64_d32", 64, 30, 61, 32, None, dict(drop_frac=0.05), {}),
    ("dos_n128_d64_cmc", 128, 20, 62, 64, CMC_AFFINE, dict(drop_frac=0.05), {}),
    ("dos_n128_noemb", 128, 20, 63, 0, None, dict(drop_frac=0.05), dict(embedding_off=True)),
    ("dos_n96_d32_awoff", 96, 20, 64, 32, None, dict(drop_frac=0.05), dict(aw_off=True)),
    ("dos_n64_dt5_iou", 64, 40, 65, 32, CMC_AFFINE, dict(drop_frac=0.15),
     dict(delta_t=5, asso_func="iou", det_thresh=0.3, min_hits=3)),
    ("dos_n256_d64", 256, 10, 66, 64, None, dict(drop_frac=0.05), {}),
]


def _deepocsort_lockstep(frames, img_shape, kw, warp, outs):
    """As _oracle_lockstep, with every padded LAP cost perturbed by 1e-6 relative noise (covers a
    float32 vs float64 embedding product, ~1e-7) and order-reversed."""
    import oracle.deepocsort as dos
    orig = dos.linear_assignment_padded
    rng = np.random.default_rng(9)

    def perturbed(cost):
        c = np.asarray(cost, np.float64)
        c = c * (1.0 + 1e-6 * rng.standard_normal(c.shape))
        m = orig(c[::-1, ::-1])
        if m.size == 0:
            return m
        m = np.stack([c.shape[0] - 1 - m[:, 0], c.shape[1] - 1 - m[:, 1]], axis=1)
        return m[np.argsort(m[:, 0])]

    exact = None
    for lap_fn in (orig, perturbed):
        dos.linear_assignment_padded = lap_fn
        try:
            t = dos.DeepOCSortOracle(**kw)
            got = [np.asarray(t.update(d, img_shape, f, warp), dtype=np.float64).reshape(-1, 8)
                   for d, f in frames]
        finally:
            dos.linear_assignment_padded = orig
        assert canonical_equal(got, outs), lap_fn.__name__
        if exact is None:
            exact = all(np.array_equal(g, o) for g, o in zip(got, outs))
    return exact


def make_g6():
    ns = refshim.load_deepocsort()
    H = refshim.Harness
    mod = ns.deep_ocsort
    out = {}
    for name, n, nf, seed, D, warp, skw, tkw in DEEPOCSORT_CASES:
        skw = dict(skw)
        skw.setdefault("low_conf_frac", 0.0)
        frames = make_frames(n, nf, seed, emb_dim=max(D, 1), **skw)
        from yolo_tracking_amd.synth import SyntheticStream
        img_shape = SyntheticStream(n, seed, emb_dim=max(D, 1), **skw).img_shape
        kw = dict(DEEPOCSORT_YAML, **tkw)
        H.high_thresh = kw["det_thresh"]
        H.warp = np.eye(2, 3) if warp is None else warp
        t = mod.DeepOCSort(None, "cpu", False, per_class=False, **kw)
        img = np.zeros((img_shape[0], img_shape[1], 3), np.uint8)
        outs, feats = [], []
        for dets, embs in frames:
            H.dets, H.feats = dets, embs
            m = dets[:, 4] > kw["det_thresh"]
            f = embs[m]
            feats.append((f / np.linalg.norm(f)) if (len(f) and D) else None)
            outs.append(np.asarray(t.update(dets, img), dtype=np.float64).reshape(-1, 8))
        exact = _deepocsort_lockstep([(d, f) for (d, _), f in zip(frames, feats)], img_shape, kw,
                                     None if warp is None else warp, outs)
        counts, rows = pack_outputs(outs)
        out[f"{name}__gen"] = np.array([n, nf, seed, D], np.int64)
        out[f"{name}__stream"] = np.array([skw["low_conf_frac"], skw.get("drop_frac", 0.0)])
        out[f"{name}__in_sum"] = np.array([float(np.sum([d.sum() for d, _ in frames])),
                                           float(np.sum([e.astype(np.float64).sum()
                                                         for _, e in frames])) if D else 0.0])
        out[f"{name}__img"] = np.array(img_shape[:2], np.int64)
        out[f"{name}__warp"] = np.asarray(H.warp, dtype=np.float64)
        out[f"{name}__params"] = np.array([kw["det_thresh"], kw["max_age"], kw["min_hits"],
                                           kw["iou_threshold"], kw["delta_t"], kw["inertia"],
                                           kw["w_association_emb"], kw["alpha_fixed_emb"],
                                           kw["aw_param"], float(kw["embedding_off"]),
                                           float(kw["cmc_off"]), float(kw["aw_off"])])
        out[f"{name}__asso"] = np.array(kw["asso_func"])
        out[f"{name}__exact"] = np.array(exact)
        out[f"{name}__out_counts"] = counts
        out[f"{name}__out"] = rows
        trk = t.trackers
        out[f"{name}__st_id"] = np.array([k.id for k in trk], np.int64)
        out[f"{name}__st_x"] = np.array([k.kf.x.ravel() for k in trk]).reshape(-1, 8)
        out[f"{name}__st_P"] = np.array([k.kf.P for k in trk]).reshape(-1, 8, 8)
        if D:
            out[f"{name}__st_emb"] = np.array([np.asarray(k.emb, np.float64) for k in trk]
                                              ).reshape(-1, D)
        print(f"G6 {name}: out_rows={len(rows)} live={len(trk)} oracle_exact={exact}")
    out["cases"] = np.array([c[0] for c in DEEPOCSORT_CASES])
    np.savez_compressed(os.path.join(HERE, "deepocsort_synth.npz"), **out)


# ------------------------------------------------------------------ G7: HybridSORT
HYBRIDSORT_YAML = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
                       asso_func="giou", inertia=0.2)                    # hybridsort.yaml
HYBRIDSORT_CASES = [  # (name, n_objects, n_frames, seed, emb_dim, stream kw, tracker kw)
    ("hs_n64_d32", 64, 30, 71, 32, dict(drop_frac=0.05), {}),
    ("hs_n128_d64", 128, 20, 72, 64, dict(drop_frac=0.05), {}),
    ("hs_n96_dt5_iou", 96, 30, 73, 32, dict(drop_frac=0.15, low_conf_frac=0.1),
     dict(delta_t=5, asso_func="iou", det_thresh=0.3, min_hits=3)),
    ("hs_n64_cls3", 64, 25, 74, 32, dict(drop_frac=0.05, n_classes=3), {}),
    ("hs_n96_diou_long", 96, 60, 75, 32, dict(drop_frac=0.3), dict(asso_func="diou", max_age=8)),
    ("hs_n256_d64", 256, 10, 76, 64, dict(drop_frac=0.05), {}),
]


def _hybridsort_lockstep(frames, kw, outs):
    """As _deepocsort_lockstep for HybridSORT (per-class calls included): the oracle must
    reproduce the reference with every padded LAP cost perturbed by 1e-6 relative noise and
    order-reversed; returns whether it matched exactly (birth order included)."""
    import oracle.hybridsort as hs
    orig = hs.linear_assignment_padded
    rng = np.random.default_rng(11)

    def perturbed(cost):
        c = np.asarray(cost, np.float64)
        c = c * (1.0 + 1e-6 * rng.standard_normal(c.shape))
        m = orig(c[::-1, ::-1])
        if m.size == 0:
            return m
        m = np.stack([c.shape[0] - 1 - m[:, 0], c.shape[1] - 1 - m[:, 1]], axis=1)
        return m[np.argsort(m[:, 0])]

    exact = None
    for lap_fn in (orig, perturbed):
        hs.linear_assignment_padded = lap_fn
        try:
            t = hs.HybridSortOracle(**kw)
            got = [np.asarray(hs.per_class_update(t, d, e), dtype=np.float64).reshape(-1, 8)
                   for d, e in frames]
        finally:
            hs.linear_assignment_padded = orig
        assert canonical_equal(got, outs), lap_fn.__name__
        if exact is None:
            exact = all(np.array_equal(g, o) for g, o in zip(got, outs))
    return exact


EMB_MARGIN = {"min": np.inf}


def make_g7():
    ns = refshim.load_hybridsort()
    H = refshim.Harness
    mod = ns.hybridsort
    asc = sys.modules["boxmot.trackers.hybridsort.association"]
    orig_assoc = asc.associate_4_points_with_score_with_reid

    def assoc_checked(*a, **k):
        # every matched pair's embedding cost must sit > 1e-6 from the correction threshold
        m, ud, ut = orig_assoc(*a, **k)
        emb = k.get("emb_cost")
        if emb is not None and emb.size:
            d = np.abs(emb - k["longterm_reid_correction_thresh"])
            EMB_MARGIN["min"] = min(EMB_MARGIN["min"], float(d.min()))
            assert d.min() > 1e-6, "embedding cost within 1e-6 of the correction threshold"
        return m, ud, ut

    mod.associate_4_points_with_score_with_reid = assoc_checked
    out = {}
    import builtins
    for name, n, nf, seed, D, skw, tkw in HYBRIDSORT_CASES:
        skw = dict(skw)
        skw.setdefault("low_conf_frac", 0.0)
        frames = make_frames(n, nf, seed, emb_dim=D, **skw)
        from yolo_tracking_amd.synth import SyntheticStream
        img_shape = SyntheticStream(n, seed, emb_dim=D, **skw).img_shape
        kw = dict(HYBRIDSORT_YAML, **tkw)
        H.match_boxes = True
        t = mod.HybridSORT(None, "cpu", False, det_thresh=kw["det_thresh"], max_age=kw["max_age"],
                           min_hits=kw["min_hits"], iou_threshold=kw["iou_threshold"],
                           delta_t=kw["delta_t"], asso_func=kw["asso_func"],
                           inertia=kw["inertia"])
        img = np.zeros((img_shape[0], img_shape[1], 3), np.uint8)
        outs = []
        pr = builtins.print
        builtins.print = lambda *a, **k: None          # the reference prints every correction
        try:
            for dets, embs in frames:
                H.dets, H.feats = dets, embs
                outs.append(np.asarray(t.update(dets, img), dtype=np.float64).reshape(-1, 8))
        finally:
            builtins.print = pr
        exact = _hybridsort_lockstep(frames, kw, outs)
        counts, rows = pack_outputs(outs)
        out[f"{name}__gen"] = np.array([n, nf, seed, D], np.int64)
        out[f"{name}__stream"] = np.array([skw["low_conf_frac"], skw.get("drop_frac", 0.0),
                                           skw.get("n_classes", 1)])
        out[f"{name}__in_sum"] = np.array([float(np.sum([d.sum() for d, _ in frames])),
                                           float(np.sum([e.astype(np.float64).sum()
                                                         for _, e in frames]))])
        out[f"{name}__params"] = np.array([kw["det_thresh"], kw["max_age"], kw["min_hits"],
                                           kw["iou_threshold"], kw["delta_t"], kw["inertia"]])
        out[f"{name}__asso"] = np.array(kw["asso_func"])
        out[f"{name}__exact"] = np.array(exact)
        out[f"{name}__out_counts"] = counts
        out[f"{name}__out"] = rows
        trk = t.trackers
        out[f"{name}__st_id"] = np.array([k.id for k in trk], np.int64)
        out[f"{name}__st_x"] = np.array([k.kf.x.ravel() for k in trk]).reshape(-1, 9)
        out[f"{name}__st_P"] = np.array([k.kf.P for k in trk]).reshape(-1, 9, 9)
        out[f"{name}__st_int"] = np.array([[k.age, k.hits, k.hit_streak, k.time_since_update,
                                            int(k.kf.observed), int(k.kf.attr_saved is not None)]
                                           for k in trk], np.int64).reshape(-1, 6)
        out[f"{name}__st_feat"] = np.array([np.asarray(k.smooth_feat, np.float32) for k in trk]
                                           ).reshape(-1, D)
        print(f"G7 {name}: out_rows={len(rows)} live={len(trk)} oracle_exact={exact} "
              f"emb_margin={EMB_MARGIN['min']:.2e}")
    out["cases"] = np.array([c[0] for c in HYBRIDSORT_CASES])
    np.savez_compressed(os.path.join(HERE, "hybridsort_synth.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["g1", "g2", "g3", "g4", "g5", "g6", "g7"]
    if "g3" in which:
        make_g3()
    if "g1" in which:
        make_g1()
    if "g2" in which:
        make_g2()
    if "g4" in which:
        make_g4()
    if "g5" in which:
        make_g5()
    if "g6" in which:
        make_g6()
    if "g7" in which:
        make_g7()
    print(f"LAP calls {TIES['calls']}, tied {TIES['ties']}")
