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


def build(out=OUT, extra=()):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    mk = open(os.path.join(CSRC, "Makefile")).read()   # every source the product builds
    names = next(l for l in mk.splitlines() if l.startswith("SRCS")).split("=", 1)[1].split()
    srcs = [os.path.join(CSRC, f) for f in names]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-ffp-contract=off", "-fno-fast-math", "-munsafe-fp-atomics", "-DYTA_STAMPS",
           *extra, "-shared", "-o", out] + srcs
    subprocess.check_call(cmd)
    print("built", out)


def show(st, base, names, title):
    t0 = st[base]
    print(f"-- {title} (block 0)")
    prev = t0
    keys = names if isinstance(names, list) else sorted(names)
    names = dict(names) if isinstance(names, list) else names
    keys = [k for k, _ in keys] if keys and isinstance(keys[0], tuple) else keys
    for k in keys:
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
    ap.add_argument("--lib", default=OUT, help="diagnostic library to build / load")
    ap.add_argument("--flags", default="", help="extra compile flags (build)")
    ap.add_argument("--tracker", choices=["bytetrack", "botsort"], default="bytetrack",
                    help="botsort: C3's engine (ReID D=512, botsort.yaml, one stream per frame)")
    args = ap.parse_args()
    if args.build:
        build(args.lib, args.flags.split())
        return
    from yolo_tracking_amd import _lib
    from yolo_tracking_amd.synth import make_frames
    lib = _lib.load_library(args.lib)
    lib.yta_debug_stamps.argtypes = [ctypes.c_void_p]
    lib.yta_debug_stamps.restype = ctypes.c_int
    _lib._lib = lib
    from yolo_tracking_amd import ByteTrackEngine
    S = args.streams
    if args.tracker == "botsort":
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from bench_tracker import BOTSORT_YAML, reid_rows
        from yolo_tracking_amd.trackers.botsort import BoTSORTEngine
        fr = make_frames(1024, args.frames, seed=5, emb_dim=512)
        eng = BoTSORTEngine(S, feat_dim=512, **BOTSORT_YAML, track_capacity=2048, max_dets=1024)
        thr = BOTSORT_YAML["track_high_thresh"]
        for f in range(args.frames):
            d, e = fr[f]
            eng.update([d] * S, [reid_rows(d, e, thr)] * S)
    else:
        base = [d for d, _ in make_frames(1024, args.frames, seed=5)]
        eng = ByteTrackEngine(S, 0.5, 0.8, 30, 30, track_capacity=2048, max_dets=1024)
        for f in range(args.frames):
            eng.update([base[f]] * S)
    st = np.zeros(128, dtype=np.uint64)
    _lib.check(lib.yta_debug_stamps(st.ctypes.data))
    st = st.astype(np.int64)
    print("stats", eng.stats())
    if args.tracker == "botsort":   # split stage 1: k_bs_prep (stage1_lists), k_bs_lap (s1_lap_body)
        show(st, 0, {2: "dets pass", 4: "tracked/lost pass"}, "k_bs_prep")
        show(st, 90, [(1, "row offsets"), (2, "CSR fill"), (8, "lap init"), (9, "lap P1 union"),
                      (10, "lap P2 roots"), (11, "lap P3 lists"), (12, "lap P4 gather"),
                      (13, "lap classify"), (14, "lap solve"), (3, "lap return"),
                      (4, "results out")], "k_bs_lap")
    elif st[60]:   # ByteTrack: stage 1 as k_s1_prep / k_s1_edges / k_s1_lap
        show(st, 60, {1: "dets pass", 2: "tracked pass", 3: "lost pass"}, "k_s1_prep")
        show(st, 66, {1: "grid build", 2: "edges"}, "k_s1_edges")
        show(st, 90, [(1, "row offsets"), (2, "CSR fill"), (8, "lap init"), (9, "lap P1 union"),
                      (10, "lap P2 roots"), (11, "lap P3 lists"), (12, "lap P4 gather"),
                      (13, "lap classify"), (14, "lap solve"), (3, "lap return"),
                      (4, "results out")], "k_s1_lap")
        print("  stage-1 LAP: n16 %d n64 %d nbig %d edges %d complex nodes %d" % tuple(st[105:110]))
    else:
        show(st, 0, STAGE1, "k_stage1")
        print("  stage-1 LAP: n16 %d n64 %d nbig %d edges %d complex nodes %d" % tuple(st[15:20]))
    show(st, 20, {4: "left/rest lists", **{k: v for k, v in STAGE1.items() if k >= 5}},
         "k_stage23 stage 2")
    show(st, 40, {1: "grid build", 2: "pass A (boxes)", 3: "pass B (features)",
                  **{k: v for k, v in STAGE1.items() if k >= 8}, 15: "end"}, "k_stage23 stage 3")
    show(st, 80, {1: "zero bits", 2: "births", 3: "expiry", 4: "t2/l2 lists", 5: "dedup grid",
                  6: "dedup queries", 7: "final lists", 8: "output rows", 9: "free list"},
         "k_finish")
    if st[126] and st[85] and st[86] and st[85] <= st[126] <= st[86]:
        print(f"  (dedup queries: tracked' boxes in {(st[126] - st[85]) / 100.0:.2f} us, the "
              f"grid queries {(st[86] - st[126]) / 100.0:.2f} us; grid {st[127] // 1000000} "
              f"cells, {st[127] % 1000000} big items; thread 0 visited {st[125]} candidates "
              f"over all frames)")
    show(st, 110, {1: "reduce", 2: "zero cells", 3: "count", 5: "cell scan", 6: "scatter"},
         "grid_build (last call)")
    # per-block timeline of the last frame's block/stream kernels
    blk = np.zeros(8 * 4096 * 2, dtype=np.uint64)
    lib.yta_debug_blocks.argtypes = [ctypes.c_void_p]
    _lib.check(lib.yta_debug_blocks(blk.ctypes.data))
    blk = blk.reshape(8, 4096, 2).astype(np.int64)[:, :S]
    print("-- per-block timeline (us; start relative to the kernel's first block start)")
    for k, name in [(0, "k_s1_prep"), (1, "k_s1_edges"), (2, "k_s1_lap"), (3, "k_stage23"),
                    (5, "k_finish")]:
        b0, b1 = blk[k, :, 0], blk[k, :, 1]
        if not b0.any():
            continue
        st0 = (b0 - b0.min()) / 100.0
        dur = (b1 - b0) / 100.0
        span = (b1.max() - b0.min()) / 100.0
        q = np.percentile(dur, [50, 90, 100])
        print(f"  {name:<11s} span {span:7.2f}  block dur p50 {q[0]:6.2f} p90 {q[1]:6.2f} max "
              f"{q[2]:6.2f}  starts: <2us {int((st0 < 2).sum())}, p50 {np.median(st0):6.2f}, "
              f"max {st0.max():6.2f}  slowest block {int(dur.argmax())}")
    # k_apply phases (blocks of the first 256 streams)
    ap = np.zeros(4096 * 5, dtype=np.uint64)
    lib.yta_debug_apply.argtypes = [ctypes.c_void_p]
    _lib.check(lib.yta_debug_apply(ap.ctypes.data))
    ap = ap.reshape(4096, 5).astype(np.int64)
    ap = ap[ap[:, 0] > 0]
    if len(ap):
        d = np.diff(ap, axis=1) / 100.0
        life = (ap[:, 4] - ap[:, 0]) / 100.0
        print(f"-- k_apply blocks sampled {len(ap)}: lifetime p50 {np.median(life):.2f} p90 "
              f"{np.percentile(life, 90):.2f} us; span {(ap[:, 4].max() - ap[:, 0].min()) / 100.0:.2f}")
        for k, name in enumerate(["level 0 (lists)", "records + det rows", "Kalman compute",
                                  "store issue"]):
            print(f"  {name:<20s} p50 {np.median(d[:, k]):6.2f}  p90 {np.percentile(d[:, k], 90):6.2f} us")


if __name__ == "__main__":
    main()
