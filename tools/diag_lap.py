#!/usr/bin/env python3
"""Diagnostic: per-phase timing of the stage-1 assignment kernel (block 0 = stream 0).

Builds a separate library with -DYTA_STAMPS (never the product build), runs the ByteTrack engine
on synthetic 1024 x 1024 frames and prints the phase spans recorded with s_memrealtime (100 MHz).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), "libyta_diag.so")
    csrc = os.path.join(REPO, "yolo_tracking_amd", "csrc")
    srcs = [os.path.join(csrc, f) for f in ("util.hip", "kat.hip", "assoc.hip", "bytetrack.hip")]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-fPIC", "-shared", "-ffp-contract=off", "-DYTA_STAMPS", "-o", out] + srcs)
    from yolo_tracking_amd import _lib
    lib = _lib.load_library(out)
    _lib._lib = lib
    lib.yta_debug_lap_stamps.argtypes = [ctypes.c_void_p]
    from yolo_tracking_amd import ByteTrackEngine
    from yolo_tracking_amd.synth import make_frames
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    frames = [[d for d, _ in make_frames(1024, 8, 50 + s)] for s in range(S)]
    eng = ByteTrackEngine(S, 0.5, 0.8, 30, 30, track_capacity=2048, max_dets=1024)
    names = ["init", "degrees", "csr-offsets", "scatter+union", "lists", "gather", "classify",
             "solve"]
    for f in range(8):
        eng.update([frames[s][f] for s in range(S)])
        st = np.zeros(16, dtype=np.uint64)
        lib.yta_debug_lap_stamps(st.ctypes.data)
        d = np.diff(st[:9].astype(np.int64)) / 100.0
        print(f"frame {f}: " + " ".join(f"{n}={v:.1f}" for n, v in zip(names, d)) +
              f" | total={(int(st[8]) - int(st[0])) / 100.0:.1f}us comps={st[10]} cnodes={st[11]} "
              f"edges={st[12]} seg16={st[13]} wave64={st[14]} big={st[15]}")


if __name__ == "__main__":
    main()
