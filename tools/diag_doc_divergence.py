#!/usr/bin/env python3
"""Debug helper (GPU box): run the DeepOCSORT engine and the oracle side by side on one stream of
a full-size golden and report the first frame where the tracker lists (ids, order, counters,
Kalman state) or the output rows differ, with the trackers involved.

    python tools/diag_doc_divergence.py [case] [full_deep|full_configs]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import full_configs as fc  # noqa: E402
from oracle.deepocsort import DeepOCSortOracle  # noqa: E402
from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "dos_n2048_cmc_f40_a"
src = sys.argv[2] if len(sys.argv) > 2 else "full_deep"
g = fc.load_deep() if src == "full_deep" else fc.load()
frames, img_shape, kw, warp, D = fc.deepocsort_frames(g, case)
eng = DeepOCSortEngine(1, feat_dim=D, **kw)
o = DeepOCSortOracle(**kw)


def ostate(o):
    t = o.trackers
    return dict(id=np.array([k.id for k in t]), age=np.array([k.age for k in t]),
                hits=np.array([k.hits for k in t]), hit_streak=np.array([k.hit_streak for k in t]),
                time_since_update=np.array([k.tsu for k in t]),
                frozen=np.array([int(k.frozen) for k in t]),
                x=np.array([k.kf.x.ravel() for k in t]).reshape(-1, 8))


t0 = time.time()
for f, (d, feats) in enumerate(frames):
    got = eng.update([d], [feats], warps=None if warp is None else warp[None],
                     img_shapes=[img_shape])[0]
    exp = np.asarray(o.update(d, img_shape, feats, warp), dtype=np.float64).reshape(-1, 8)
    a, b = eng.state(0), ostate(o)
    bad = []
    if not np.array_equal(a["id"], b["id"]):
        bad.append("ids")
    else:
        for k in ("age", "hits", "hit_streak", "time_since_update", "frozen"):
            if not np.array_equal(a[k], b[k]):
                bad.append(k)
        dx = np.abs(a["x"] - b["x"]) / np.maximum(1.0, np.abs(b["x"]))
        if dx.max() > 1e-9:
            bad.append(f"x (max rel {dx.max():.3g} at tracker {int(np.argmax(dx.max(1)))})")
    same_rows = got.shape == exp.shape and np.array_equal(got[:, 4:], exp[:, 4:])
    print(f"frame {f}: rows gpu {len(got)} ref {len(exp)} rows_equal={same_rows} "
          f"state_diff={bad} ({time.time() - t0:.0f}s)", flush=True)
    if bad or not same_rows:
        ga, gb = set(a["id"].tolist()), set(b["id"].tolist())
        print(" trackers only-gpu", sorted(ga - gb)[:20], "only-ref", sorted(gb - ga)[:20])
        ra, rb = set(got[:, 4].astype(int).tolist()), set(exp[:, 4].astype(int).tolist())
        print(" out ids only-gpu", sorted(ra - rb)[:20], "only-ref", sorted(rb - ra)[:20])
        ids = sorted((ga ^ gb) | (ra ^ rb))[:6]
        if not ids and "ids" not in bad:
            for k in ("age", "hits", "hit_streak", "time_since_update", "frozen"):
                w = np.nonzero(a[k] != b[k])[0]
                if len(w):
                    ids = [int(a["id"][i]) for i in w[:6]]
                    break
        for tid in ids:
            for name, st in (("gpu", a), ("ref", b)):
                w = np.nonzero(st["id"] == tid)[0]
                if len(w):
                    i = int(w[0])
                    print(f"  {name} id {tid} pos {i}: age {st['age'][i]} hits {st['hits'][i]} "
                          f"streak {st['hit_streak'][i]} tsu {st['time_since_update'][i]} "
                          f"frozen {st['frozen'][i]} x {np.array2string(st['x'][i], precision=6)}")
                else:
                    print(f"  {name} id {tid}: absent")
            for name, rows in (("gpu", got), ("ref", exp)):
                w = np.nonzero(rows[:, 4] == tid)[0]
                print(f"  {name} row id {tid}:", rows[w[0]] if len(w) else "none")
        break
else:
    print("no divergence")
