"""SparseOptFlow camera-motion estimation throughput: S camera streams, one
BGR frame per stream per step (default 1920x1080, the MOT17 frame size), estimator scale 0.1 as in
sof.py; frames and detection boxes resident in HBM; one yta_sof_apply_device call per step (all
streams' frames in the same 5 launches), warps left on the device.  Frame 0 is the first-frame
path (goodFeaturesToTrack); the timed steps are the steady state (pyramids, Lucas-Kanade of the
stored corners, RANSAC + LM).  Frames: a textured scene per stream seen through a moving crop
window (integer shifts of a few px per frame).  CPU leg: oracle/cmc_sof.py (NumPy restatement) on
one stream, 1 thread, a bounded sample of the same frames.  Prints one JSON line.
--estimator ecc: the ECC estimator instead (ecc.py, csrc/ecc.hip: one yta_ecc_apply_device call
per step, warp_mode --warp-mode, default euclidean), its CPU leg oracle/cmc_ecc.py."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def frames_for(S, F, H, W, seed):
    """[F][S] frames: stream s crops an (H + 8F) x (W + 8F) scene at (4f + s % 3, 2f)."""
    from cmc_frames import bgr, scene
    out = np.empty((F, S, H, W, 3), np.uint8)
    base = [bgr(scene((H + 8 * F) // 4, (W + 8 * F) // 4, seed + s % 4), s) for s in range(min(S, 4))]
    for s in range(S):
        big = np.repeat(np.repeat(base[s % len(base)], 4, axis=0), 4, axis=1)
        for f in range(F):
            y, x = 2 * f, 4 * f + s % 3
            out[f, s] = big[y:y + H, x:x + W]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--dets", type=int, default=32)
    ap.add_argument("--scale", type=float, default=0.1)
    ap.add_argument("--cpu-frames", type=int, default=4)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--estimator", choices=["sof", "ecc"], default="sof")
    ap.add_argument("--warp-mode", type=int, default=1, help="ECC: 0 translation, 1 euclidean, 2 affine")
    args = ap.parse_args()
    import torch
    from yolo_tracking_amd import _lib
    from yolo_tracking_amd.motion.sof import SofEngine
    S, H, W, F = args.streams, args.h, args.w, args.steps + 2
    t0 = time.time()
    fr = frames_for(S, F, H, W, 3)
    rng = np.random.default_rng(1)
    xy = rng.uniform(0, 1, (S, args.dets, 2)) * [W - 200, H - 300]
    wh = rng.uniform(40, 200, (S, args.dets, 2))
    dets = np.concatenate([xy, xy + wh], 2).reshape(-1, 4)
    gen_s = time.time() - t0
    d = torch.device("cuda", 0)
    d_fr = torch.from_numpy(fr.reshape(F, -1)).to(d)
    d_off = torch.arange(S, dtype=torch.int64, device=d) * (H * W * 3)
    d_hw = torch.tensor([H, W] * S, dtype=torch.int32, device=d)
    d_dets = torch.from_numpy(dets).to(d)
    d_doff = torch.arange(S + 1, dtype=torch.int32, device=d) * args.dets
    ecc = args.estimator == "ecc"
    d_warps = torch.zeros((S, 6), dtype=torch.float32 if ecc else torch.float64, device=d)
    hs = ctypes.c_void_p()
    if ecc:
        from yolo_tracking_amd.motion.ecc import EccEngine
        eng = EccEngine(S, args.warp_mode, 1e-5, 100, args.scale, 0, H, W)
        lib = eng.lib
        _lib.check(lib.yta_ecc_hip_stream(eng.handle, ctypes.byref(hs)))
    else:
        eng = SofEngine(S, args.scale, 0, H, W)
        lib = eng.lib
        _lib.check(lib.yta_sof_hip_stream(eng.handle, ctypes.byref(hs)))
    stream = torch.cuda.ExternalStream(hs.value, device=d)
    sync = (lambda: _lib.check(lib.yta_ecc_sync(eng.handle))) if ecc else \
        (lambda: _lib.check(lib.yta_sof_sync(eng.handle)))

    def step(f):
        if ecc:
            _lib.check(lib.yta_ecc_apply_device(
                eng.handle, ctypes.c_void_p(d_fr[f].data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
                ctypes.c_void_p(d_hw.data_ptr()), ctypes.c_void_p(d_warps.data_ptr())))
            return
        _lib.check(lib.yta_sof_apply_device(
            eng.handle, ctypes.c_void_p(d_fr[f].data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
            ctypes.c_void_p(d_hw.data_ptr()), ctypes.c_void_p(d_dets.data_ptr()), 4,
            ctypes.c_void_p(d_doff.data_ptr()), ctypes.c_void_p(d_warps.data_ptr())))

    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record(stream)
    step(0)                            # first frame: corners
    e[1].record(stream)
    step(1)                            # warm-up of the steady-state path
    sync()
    t1 = time.perf_counter()
    e[2].record(stream)
    for f in range(2, F):
        step(f)
    e_end = torch.cuda.Event(enable_timing=True)
    e_end.record(stream)
    sync()
    wall = time.perf_counter() - t1
    torch.cuda.synchronize()
    first_ms = e[0].elapsed_time(e[1])
    steady_ms = e[2].elapsed_time(e_end) / (F - 2)
    if ecc:
        oc, iters, _ = eng.outcome()
        extra = {"iters_mean": float(np.mean(iters)), "iters_max": int(np.max(iters)),
                 "warp_mode": args.warp_mode}
    else:
        oc = eng.outcome()
        extra = {"corners_stream0_3": [len(eng.state(s)["keypoints"]) for s in range(min(S, 4))]}
    name = "ECC.apply()" if ecc else "SparseOptFlow.apply()"
    line = {"metric": f"{name} frames/s", "value": S / (steady_ms * 1e-3),
            "unit": "frames/s", "streams": S, "frame": f"{W}x{H}", "scale": args.scale,
            "steps": F - 2, "ms_per_step": steady_ms, "first_frame_ms": first_ms,
            "wall_ms_per_step": 1000 * wall / (F - 2), "outcomes": np.bincount(oc, minlength=3).tolist(),
            "dets_per_stream": args.dets, "gen_s": round(gen_s, 1),
            "data": "synthetic textured scene, moving crop window", **extra}
    if not args.no_cpu and ecc:
        from oracle import cmc_ecc as ce
        o = ce.ECCOracle(warp_mode=args.warp_mode, scale=args.scale)
        o.apply(fr[0, 0])
        o.apply(fr[1, 0])
        n = min(args.cpu_frames, F - 2)
        c0 = time.perf_counter()
        for f in range(2, 2 + n):
            o.apply(fr[f, 0])
        cpu_s = (time.perf_counter() - c0) / n
        line["cpu_baseline"] = {"value": 1.0 / cpu_s, "unit": "frames/s", "cores": 1,
                                "kind": "port",
                                "sample": f"oracle/cmc_ecc.py, stream 0, frames 2..{1 + n}, "
                                          f"{cpu_s * 1000:.1f} ms/frame, 1 thread"}
    elif not args.no_cpu:
        from oracle import cmc_sof as cs
        o = cs.SparseOptFlowOracle(args.scale)
        dd = dets[:args.dets]
        o.apply(fr[0, 0], dd)
        o.apply(fr[1, 0], dd)
        n = min(args.cpu_frames, F - 2)
        c0 = time.perf_counter()
        for f in range(2, 2 + n):
            o.apply(fr[f, 0], dd)
        cpu_s = (time.perf_counter() - c0) / n
        line["cpu_baseline"] = {"value": 1.0 / cpu_s, "unit": "frames/s", "cores": 1,
                                "kind": "port",
                                "sample": f"oracle/cmc_sof.py, stream 0, frames 2..{1 + n}, "
                                          f"{cpu_s * 1000:.1f} ms/frame, 1 thread"}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
