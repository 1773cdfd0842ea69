#!/usr/bin/env python3
"""Diagnostic: phase stamps of stream 0 inside k_ocsort (and its dense LAP).

    python tools/diag_ocsort.py --build     # (CPU) tools/_diag/libyta_oc_diag.so with -DYTA_STAMPS
    python tools/diag_ocsort.py [--n 256]   # (GPU) run frames, print the last frame's phases (us)
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
CSRC = os.path.join(REPO, "yolo_tracking_amd", "csrc")
OUT = os.path.join(REPO, "tools", "_diag", "libyta_oc_diag.so")
NAMES = {1: "A predict", 2: "B columns", 43: "E counts", 60: "lap colreduce",
         61: "lap transfer", 62: "lap rowreduce", 63: "lap augment", 44: "E lap/fast",
         45: "E lists", 46: "F byte", 47: "G ocr", 48: "H updates", 49: "I births",
         50: "J outputs"}


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in ("util.hip", "kat.hip", "bytetrack.hip", "ocsort.hip")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-ffp-contract=off", "-fno-fast-math", "-munsafe-fp-atomics", "-DYTA_STAMPS",
           "-shared", "-o", OUT] + srcs
    subprocess.check_call(cmd)
    print("built", OUT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--frames", type=int, default=12)
    args = ap.parse_args()
    if args.build:
        build()
        return
    os.environ["YTA_LIBRARY"] = OUT
    from yolo_tracking_amd import _lib
    from yolo_tracking_amd.synth import SyntheticStream, make_frames
    from yolo_tracking_amd.trackers.ocsort import OCSortEngine
    lib = _lib.load_library()
    lib.yta_ocsort_debug_stamps.argtypes = [ctypes.c_void_p]
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, asso_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2, use_byte=False)
    fr = [d for d, _ in make_frames(args.n, args.frames, 2000, low_conf_frac=0.0)]
    shape = SyntheticStream(args.n, 2000, low_conf_frac=0.0).img_shape
    eng = OCSortEngine(1, **kw, track_capacity=2 * args.n, max_dets=args.n)
    st = (ctypes.c_ulonglong * 128)()
    for f, d in enumerate(fr):
        eng.update([d], [shape])
    lib.yta_ocsort_debug_stamps(st)
    print("  counts over all frames: rowreduce iters", st[120], "augmentations", st[121],
          "gathers", st[122], "scans", st[123], "register sweeps", st[124])
    print("  augment time over all frames (us): row staging", st[110] / 100.0, "relax sweeps",
          st[111] / 100.0, "gathers", st[112] / 100.0)
    print(f"  pre kernel: {(st[2] - st[0]) / 100.0:.2f} us (A {(st[1] - st[0]) / 100.0:.2f})")
    t0 = st[40]
    prev = t0
    order = [43, 60, 61, 62, 63, 44, 45, 46, 47, 48, 49, 50]
    for k in order:
        v = st[k]
        if v == 0 or v < prev:
            continue
        print(f"  {NAMES[k]:<16s} {(v - prev) / 100.0:10.2f} us   (t={(v - t0) / 100.0:9.2f})")
        prev = v
    print(eng.stats())


if __name__ == "__main__":
    main()
