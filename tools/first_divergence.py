#!/usr/bin/env python3
"""Debug helper: run the GPU engine and the oracle side by side on one MOT17-mini sequence and
report the first frame where the tracked / lost lists (ids, order, state) differ."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import mot_frames  # noqa: E402
from oracle.bytetrack import ByteTrackOracle  # noqa: E402
from yolo_tracking_amd import ByteTrackEngine  # noqa: E402

seq = sys.argv[1] if len(sys.argv) > 1 else "MOT17_02_FRCNN"
g = np.load(os.path.join(REPO, "tests", "golden", "bytetrack_mot17.npz"))
eng = ByteTrackEngine(1, 0.5, 0.8, 30, 30)
ref = ByteTrackOracle(0.5, 0.8, 30, 30)
for f, d in enumerate(mot_frames(g, seq)):
    eng.update([d])
    ref.update(d)
    st = eng.state(0)
    got_t = list(st["id"][st["list"] == 0])
    got_l = list(st["id"][st["list"] == 1])
    exp_t = [t.track_id for t in ref.tracked]
    exp_l = [t.track_id for t in ref.lost]
    if got_t != exp_t or got_l != exp_l:
        print("first divergence at frame", f)
        print(" tracked only-gpu", sorted(set(got_t) - set(exp_t)), "only-ref",
              sorted(set(exp_t) - set(got_t)))
        print(" lost only-gpu", sorted(set(got_l) - set(exp_l)), "only-ref",
              sorted(set(exp_l) - set(got_l)))
        print(" lost gpu", got_l)
        print(" lost ref", exp_l)
        break
else:
    print("no divergence")
