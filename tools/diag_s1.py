#!/usr/bin/env python3
"""Diagnostic: per-phase stamps (block 0) of ByteTrack's split stage 1 (k_s1_prep / k_s1_edges /
k_s1_lap) and of k_stage23 / k_finish, from the -DYTA_STAMPS library that tools/diag_stamps.py
--build compiles.   python tools/diag_s1.py [--streams 1024] [--frames 25]   (GPU)"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from diag_stamps import OUT  # noqa: E402


def show(st, base, names, title):
    """names: {stamp index: phase} in the order the phases run."""
    t0 = prev = st[base]
    print(f"-- {title} (block 0)")
    for k, name in names.items():
        v = st[base + k]
        if v == 0 or v < prev:
            continue
        print(f"  {name:<22s} {(v - prev) / 100.0:8.2f} us   (t={(v - t0) / 100.0:7.2f})")
        prev = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=25)
    args = ap.parse_args()
    from yolo_tracking_amd import _lib
    from yolo_tracking_amd.synth import make_frames
    lib = _lib.load_library(OUT)
    lib.yta_debug_stamps.argtypes = [ctypes.c_void_p]
    lib.yta_debug_stamps.restype = ctypes.c_int
    _lib._lib = lib
    from yolo_tracking_amd import ByteTrackEngine
    S = args.streams
    frames = [make_frames(1024, args.frames, seed=1000 + q) for q in range(4)]
    eng = ByteTrackEngine(S, 0.5, 0.8, 30, 30, track_capacity=2048, max_dets=1024)
    for f in range(args.frames):
        eng.update([frames[q % 4][f][0] for q in range(S)])
    st = np.zeros(128, dtype=np.uint64)
    _lib.check(lib.yta_debug_stamps(st.ctypes.data))
    st = st.astype(np.int64)
    print("stats", eng.stats())
    show(st, 60, {1: "dets pass", 2: "tracked pass", 3: "lost pass + counters"}, "k_s1_prep")
    show(st, 66, {1: "grid build", 2: "pool queries"}, "k_s1_edges")
    show(st, 90, {1: "row offsets", 2: "csr fill", 8: "lap init", 9: "lap P1 union",
                  10: "lap P2 roots", 11: "lap P3 lists", 12: "lap P4 gather",
                  13: "lap classify", 14: "lap solve", 3: "lap end", 4: "write out"}, "k_s1_lap")
    print("  LAP: n16 %d n64 %d nbig %d edges %d complex nodes %d" % tuple(st[105:110]))
    print("  shapes (all LAP calls of block 0): k2l1 %d k3+l1 %d k2l2 %d k2l3+ %d k3l2 %d "
          "other<=6 %d bigger %d" % tuple(st[117:124]))
    show(st, 80, {1: "zero bits", 2: "births", 3: "expiry", 4: "t2/l2 lists", 5: "dedup grid",
                  6: "dedup queries", 7: "final lists", 8: "output rows", 9: "free list"},
         "k_finish")


if __name__ == "__main__":
    main()
