#!/usr/bin/env python3
"""Diagnostic: per-phase wall-clock stamps of block 0 inside the stage kernels.

    python tools/diag_stamps.py --build          # (CPU) compile tools/_diag/libyta_diag.so
    python tools/diag_stamps.py [--streams 256]  # (GPU) run frames, print phase durations (us)

The diagnostic library is the product sources compiled with -DYTA_STAMPS (s_memrealtime, 100 MHz,
thread 0 of block 0 after each phase's barrier); it is never loaded by the package itself.
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
OUT = os.path.join(REPO, "tools", "_diag", "libyta_diag.so")

STAGE1 = {2: "dets pass", 4: "tracked/lost pass",
          5: "grid build", 6: "edges pass 1", 7: "edges pass 2", 8: "lap init", 9: "lap P1 union",
          10: "lap P2 roots", 11: "lap P3 lists", 12: "lap P4 gather", 13: "lap classify",
          14: "lap solve"}


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    mk = open(os.path.join(CSRC, "Makefile")).read()   # every source the product builds
    names = next(l for l in mk.splitlines() if l.startswith("SRCS")).split("=", 1)[1].split()
    srcs = [os.path.join(CSRC, f) for f in names]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-ffp-contract=off", "-fno-fast-math", "-munsafe-fp-atomics", "-DYTA_STAMPS",
           "-shared", "-o", OUT] + srcs
    subprocess.check_call(cmd)
    print("built", OUT)


def show(st, base, names, title):
    t0 = st[base]
    print(f"-- {title} (block 0)")
    prev = t0
    for k in sorted(names):
        v = st[base + k]
        if v == 0 or v < prev:
            continue
        print(f"  {names[k]:<22s} {(v - prev) / 100.0:8.2f} us   (t={(v - t0) / 100.0:7.2f})")
        prev = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--frames", type=int, default=6)
    args = ap.parse_args()
    if args.build:
        build()
        return
    from yolo_tracking_amd import _lib
    from yolo_tracking_amd.synth import make_frames
    lib = _lib.load_library(OUT)
    lib.yta_debug_stamps.argtypes = [ctypes.c_void_p]
    lib.yta_debug_stamps.restype = ctypes.c_int
    _lib._lib = lib
    from yolo_tracking_amd import ByteTrackEngine
    S = args.streams
    base = [d for d, _ in make_frames(1024, args.frames, seed=5)]
    eng = ByteTrackEngine(S, 0.5, 0.8, 30, 30, track_capacity=2048, max_dets=1024)
    for f in range(args.frames):
        eng.update([base[f]] * S)
    st = np.zeros(128, dtype=np.uint64)
    _lib.check(lib.yta_debug_stamps(st.ctypes.data))
    st = st.astype(np.int64)
    print("stats", eng.stats())
    show(st, 0, STAGE1, "k_stage1")
    print("  stage-1 LAP: n16 %d n64 %d nbig %d edges %d complex nodes %d" % tuple(st[15:20]))
    show(st, 20, {4: "left/rest lists", **{k: v for k, v in STAGE1.items() if k >= 5}},
         "k_stage23 stage 2")
    show(st, 40, {k: v for k, v in STAGE1.items() if k >= 5}, "k_stage23 stage 3")
    show(st, 80, {1: "zero bits", 2: "births", 3: "expiry", 4: "t2/l2 lists", 5: "dedup grid",
                  6: "dedup queries", 7: "final lists", 8: "output rows", 9: "free list"},
         "k_finish")
    show(st, 110, {1: "reduce", 2: "zero cells", 3: "count", 5: "cell scan", 6: "scatter"},
         "grid_build (last call)")


if __name__ == "__main__":
    main()
