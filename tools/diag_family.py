#!/usr/bin/env python3
"""Diagnostic: phase stamps of stream 0's association kernel (DeepOCSORT / HybridSORT) and the
rectangular solver's counters for the last frame.

    python tools/diag_family.py --build                      # (CPU) tools/_diag/libyta_diag.so
    python tools/diag_family.py --tracker hybridsort --n 4096 --frames 8   # (GPU)
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
PHASES = {"deepocsort": ["first round", "lists", "OCR", "updates", "births", "outputs"],
          "hybridsort": ["first-round LAP", "lists / correction", "updates", "OCR", "misses",
                         "births", "outputs"]}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--tracker", choices=["deepocsort", "hybridsort"], default="hybridsort")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=8)
    args = ap.parse_args()
    if args.build:
        build()
        return
    os.environ["YTA_LIBRARY"] = OUT
    from yolo_tracking_amd import _lib
    from yolo_tracking_amd.synth import SyntheticStream, make_frames
    lib = _lib.load_library()
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2)
    fr = make_frames(args.n, args.frames, 2000, emb_dim=512, low_conf_frac=0.0)
    feats = [(e / np.linalg.norm(e)).astype(np.float32) for _, e in fr]
    if args.tracker == "hybridsort":
        from yolo_tracking_amd.trackers.hybridsort import HybridSortEngine
        eng = HybridSortEngine(1, feat_dim=512, **kw, track_capacity=2 * args.n, max_dets=args.n)
        stamps = lib.yta_hybridsort_debug_stamps
        step = lambda f: eng.update([fr[f][0]], [feats[f]])
    else:
        from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine
        eng = DeepOCSortEngine(1, feat_dim=512, **kw, track_capacity=2 * args.n, max_dets=args.n)
        shape = SyntheticStream(args.n, 2000, emb_dim=512, low_conf_frac=0.0).img_shape
        warp = np.array([[[1.0, 1e-3, 0.5], [-1e-3, 1.0, -0.3]]])
        stamps = lib.yta_deepocsort_debug_stamps
        step = lambda f: eng.update([fr[f][0]], [feats[f]], warp, [shape])
    stamps.argtypes = [ctypes.c_void_p]
    a = (ctypes.c_ulonglong * 128)()
    b = (ctypes.c_ulonglong * 128)()
    for f in range(args.frames - 1):
        step(f)
    stamps(a)
    step(args.frames - 1)
    stamps(b)
    d = lambda k: b[k] - a[k]
    print(f"last frame: augmentations {d(100)}, solver steps {d(101)}, relax {d(102) / 100:.1f} us,"
          f" reduce {d(103) / 100:.1f} us, solver total {(b[105] - b[104]) / 100:.1f} us")
    t0 = b[40]
    prev = t0
    for k, name in enumerate(PHASES[args.tracker], start=1):
        v = b[40 + k]
        if v >= prev:
            print(f"  {name:<20s} {(v - prev) / 100:10.1f} us")
            prev = v
    print(f"  {'rest':<20s} {(b[47] - prev) / 100:10.1f} us   (kernel {(b[47] - t0) / 100:.1f} us)")
    print(eng.stats())


if __name__ == "__main__":
    main()
