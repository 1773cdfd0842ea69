#!/usr/bin/env python3
"""Debug helper: the engine's duplicate-removal inputs / flags at one MOT17-02 frame."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import mot_frames  # noqa: E402
from oracle import geometry  # noqa: E402
from yolo_tracking_amd import ByteTrackEngine, _lib  # noqa: E402

g = np.load(os.path.join(REPO, "tests", "golden", "bytetrack_mot17.npz"))
frames = mot_frames(g, "MOT17_02_FRCNN")
eng = ByteTrackEngine(1, 0.5, 0.8, 30, 30)
last = int(sys.argv[1]) if len(sys.argv) > 1 else 316
for f in range(last):
    eng.update([frames[f]])
cap, _ = eng.capacity()
nt, nl = ctypes.c_int(), ctypes.c_int()
tb, lb = np.zeros((cap, 4)), np.zeros((cap, 4))
ages, drops = np.zeros(2 * cap, np.int32), np.zeros(2 * cap, np.int32)
_lib.check(eng.lib.yta_bytetrack_debug_dedup(eng.handle, 0, ctypes.byref(nt), ctypes.byref(nl),
                                             tb.ctypes.data, lb.ctypes.data, ages.ctypes.data,
                                             drops.ctypes.data))
nt, nl = nt.value, nl.value
T, L = tb[:nt], lb[:nl]
d = 1 - geometry.iou_batch(T, L)
for p, q in zip(*np.nonzero(d < 0.15)):
    print("dup pair", p, q, "dist", d[p, q], "ages", ages[p], ages[nt + q], "drops", drops[p],
          drops[nt + q])
print("n_t2", nt, "n_l2", nl, "dropA sum", drops[:nt].sum(), "dropB sum", drops[nt:nt + nl].sum())
print("grid pairs", _lib.grid_pairs(T, L, 0.15))
