#!/usr/bin/env python3
"""Debug helper: state of two tracks after a given MOT17-02 frame (GPU engine vs oracle)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import mot_frames  # noqa: E402
from oracle import geometry  # noqa: E402
from oracle.bytetrack import ByteTrackOracle  # noqa: E402
from yolo_tracking_amd import ByteTrackEngine  # noqa: E402

g = np.load(os.path.join(REPO, "tests", "golden", "bytetrack_mot17.npz"))
frames = mot_frames(g, "MOT17_02_FRCNN")
eng = ByteTrackEngine(1, 0.5, 0.8, 30, 30)
ref = ByteTrackOracle(0.5, 0.8, 30, 30)
last = int(sys.argv[1]) if len(sys.argv) > 1 else 316
for f in range(last):
    eng.update([frames[f]])
    ref.update(frames[f])
st = eng.state(0)
for tid in (42, 50):
    k = np.nonzero(st["id"] == tid)[0]
    if len(k):
        k = k[0]
        m = st["mean"][k]
        w = m[2] * m[3]
        box = np.array([m[0] - w / 2, m[1] - m[3] / 2, m[0] + w / 2, m[1] + m[3] / 2])
        print("gpu", tid, "list", st["list"][k], "state", st["state"][k], "frame", st["frame_id"][k],
              "start", st["start_frame"][k], "box", box)
for t in ref.tracked + ref.lost:
    if t.track_id in (42, 50):
        print("ref", t.track_id, "state", t.state, "frame", t.frame_id, "start", t.start_frame,
              "box", t.box())
a = [t for t in ref.tracked if t.track_id == 42]
print("cap/maxd", eng.capacity())
