"""Loaders for the full-size goldens (tests/golden/full_configs.npz, made by
tests/golden/make_goldens_full.py from the reference): inputs regenerated from their seeds with
yolo_tracking_amd.synth and checked against the stored checksums, per-frame outputs checked
against SHA-256 digests of the reference's rows (plus the last frame in full)."""
import hashlib
import os

import numpy as np

from yolo_tracking_amd.synth import make_frames

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "golden", "full_configs.npz")
DOS_CMC = ["dos_n2048_d512_cmc_a", "dos_n2048_d512_cmc_b", "dos_n2048_d512_cmc_c",
           "dos_n2048_d512_cmc_d"]
HS_4096 = ["hs_n4096_d512_a", "hs_n4096_d512_b"]
# long cases (tests/golden/make_goldens_deep.py -> full_deep.npz)
DEEP_PATH = os.path.join(HERE, "golden", "full_deep.npz")
DOS_F40 = ["dos_n2048_cmc_f40_a", "dos_n2048_cmc_f40_b"]
HS_S8 = [f"hs_n4096_s8_{k}" for k in "abcdefgh"]


def load():
    return np.load(PATH)


def load_deep():
    return np.load(DEEP_PATH)


def digest(rows):
    a = np.ascontiguousarray(np.asarray(rows, dtype="<f8").reshape(-1, 8))
    return hashlib.sha256(a.tobytes()).digest()


def check_frame(g, name, f, rows):
    """One frame of one stream against the reference: row count, digest, the last frame's rows in full."""
    rows = np.asarray(rows, dtype=np.float64).reshape(-1, 8)
    counts = g[f"{name}__out_counts"]
    assert len(rows) == counts[f], (name, f, len(rows), int(counts[f]))
    if f == len(counts) - 1:
        assert np.array_equal(rows, g[f"{name}__out_last"]), (name, f)
    assert digest(rows) == bytes(g[f"{name}__out_sha"][f]), (name, f)


def check_frame_close(g, name, f, rows, rtol=1e-9, atol=1e-9):
    """For the CPU oracle (boxes agree with the reference's to 1e-9 relative, not bit for bit):
    row count, every frame's ids and det_ind exactly, the last frame's rows to rtol."""
    rows = np.asarray(rows, dtype=np.float64).reshape(-1, 8)
    counts = g[f"{name}__out_counts"]
    assert len(rows) == counts[f], (name, f, len(rows), int(counts[f]))
    off = int(np.sum(counts[:f]))
    idx = g[f"{name}__out_idx"][off:off + counts[f]]
    assert np.array_equal(rows[:, [4, 7]].astype(np.int64), idx), (name, f)
    if f == len(counts) - 1:
        exp = g[f"{name}__out_last"]
        assert np.array_equal(rows[:, 4:], exp[:, 4:]), (name, f)
        np.testing.assert_allclose(rows[:, :4], exp[:, :4], rtol=rtol, atol=atol)


def bytetrack_frames(g, name):
    n, nf, seed = (int(x) for x in g[f"{name}__gen"])
    frames = [d for d, _ in make_frames(n, nf, seed)]
    assert float(np.sum([d.sum() for d in frames])) == g[f"{name}__in_sum"][0]
    return frames


def botsort_frames(g, name):
    """(frames [(dets, embs)], params dict, D) of the full-size BoT-SORT case."""
    n, nf, seed, D = (int(x) for x in g[f"{name}__gen"])
    skw = {}
    if f"{name}__stream" in g.files:
        low, drop = (float(x) for x in g[f"{name}__stream"])
        skw = dict(low_conf_frac=low, drop_frac=drop)
    frames = make_frames(n, nf, seed, emb_dim=D, **skw)
    sums = g[f"{name}__in_sum"]
    assert float(np.sum([d.sum() for d, _ in frames])) == sums[0]
    assert float(np.sum([e.astype(np.float64).sum() for _, e in frames])) == sums[1]
    p = g[f"{name}__params"]
    params = dict(track_high_thresh=p[0], track_low_thresh=p[1], new_track_thresh=p[2],
                  track_buffer=int(p[3]), match_thresh=p[4], proximity_thresh=p[5],
                  appearance_thresh=p[6], frame_rate=int(p[7]),
                  fuse_first_associate=bool(p[8]), with_reid=bool(p[9]))
    return frames, params, D


def deepocsort_frames(g, name):
    """(frames [(dets, feats)], img_shape, kwargs, warp or None, D) of a full-size DeepOCSORT
    case (the surge case appends a second population from frame 2 on)."""
    n, nf, seed, D = (int(x) for x in g[f"{name}__gen"])
    low, drop = (float(x) for x in g[f"{name}__stream"])
    raw = make_frames(n, nf, seed, emb_dim=D, low_conf_frac=low, drop_frac=drop)
    if f"{name}__seed2" in g.files:
        b = make_frames(n, nf, int(g[f"{name}__seed2"]), emb_dim=D, low_conf_frac=low,
                        drop_frac=drop)
        raw = [raw[0]] + [(np.concatenate([raw[f][0], b[f][0]]),
                           np.concatenate([raw[f][1], b[f][1]])) for f in range(1, nf)]
    sums = g[f"{name}__in_sum"]
    assert float(np.sum([d.sum() for d, _ in raw])) == sums[0]
    assert float(np.sum([e.astype(np.float64).sum() for _, e in raw])) == sums[1]
    p = g[f"{name}__params"]
    kw = dict(det_thresh=float(p[0]), max_age=int(p[1]), min_hits=int(p[2]),
              iou_threshold=float(p[3]), delta_t=int(p[4]), inertia=float(p[5]),
              w_association_emb=float(p[6]), alpha_fixed_emb=float(p[7]), aw_param=float(p[8]),
              embedding_off=bool(p[9]), cmc_off=bool(p[10]), aw_off=bool(p[11]),
              asso_func=str(g[f"{name}__asso"]))
    frames = []
    for d, e in raw:
        f = e[d[:, 4] > kw["det_thresh"]]
        frames.append((d, f / np.linalg.norm(f)))
    warp = g[f"{name}__warp"]
    warp = None if np.array_equal(warp, np.eye(2, 3)) else warp
    return frames, tuple(int(v) for v in g[f"{name}__img"]), kw, warp, D


def hybridsort_frames(g, name):
    """(frames [(dets, raw embeddings)], kwargs, D) of a full-size HybridSORT case."""
    n, nf, seed, D = (int(x) for x in g[f"{name}__gen"])
    low, drop, ncls = (float(x) for x in g[f"{name}__stream"])
    raw = make_frames(n, nf, seed, emb_dim=D, low_conf_frac=low, drop_frac=drop,
                      n_classes=int(ncls))
    sums = g[f"{name}__in_sum"]
    assert float(np.sum([d.sum() for d, _ in raw])) == sums[0]
    assert float(np.sum([e.astype(np.float64).sum() for _, e in raw])) == sums[1]
    p = g[f"{name}__params"]
    kw = dict(det_thresh=float(p[0]), max_age=int(p[1]), min_hits=int(p[2]),
              iou_threshold=float(p[3]), delta_t=int(p[4]), inertia=float(p[5]),
              asso_func=str(g[f"{name}__asso"]))
    return raw, kw, D
