#!/usr/bin/env python3
"""Experiment: S ByteTrack streams split over E engines (each with its own HIP stream) so that
one engine's latency-bound stage kernels overlap another's HBM-bound k_apply / k_finish.

    python tools/bench_engines.py --streams 1024 --engines 2 [--steps 20]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1024)
    ap.add_argument("--engines", type=int, default=2)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1000)
    a = ap.parse_args()
    import torch
    from yolo_tracking_amd import ByteTrackEngine, _lib
    S, N, E = a.streams, a.n, a.engines
    F = a.warmup + a.steps
    per_stream = [bench.gen_stream_frames(N, F, sd) for sd in bench.stream_seeds(a.seed, 0, S)]
    Se = S // E
    engs = []
    for e in range(E):
        ss = per_stream[e * Se:(e + 1) * Se]
        host = np.stack([np.concatenate([ss[s][f] for s in range(Se)]) for f in range(F)])
        off = np.array([[sum(len(ss[q][f]) for q in range(s)) for s in range(Se + 1)]
                        for f in range(F)], dtype=np.int32)
        eng = ByteTrackEngine(Se, 0.5, 0.8, 30, 30, device=0, track_capacity=2 * N, max_dets=N)
        cap, _ = eng.capacity()
        engs.append(dict(eng=eng, d=torch.from_numpy(host).cuda(), o=torch.from_numpy(off).cuda(),
                         out=torch.empty((Se * cap, 8), dtype=torch.float64, device="cuda"),
                         cnt=torch.zeros(Se, dtype=torch.int32, device="cuda"),
                         rb=N * 6 * 8 * Se))

    def step(f):
        for x in engs:
            _lib.check(x["eng"].lib.yta_bytetrack_update_device(
                x["eng"].handle, ctypes.c_void_p(x["d"].data_ptr() + f * x["rb"]),
                ctypes.c_void_p(x["o"].data_ptr() + f * (Se + 1) * 4),
                ctypes.c_void_p(x["out"].data_ptr()), ctypes.c_void_p(x["cnt"].data_ptr())))

    def sync():
        for x in engs:
            _lib.check(x["eng"].lib.yta_bytetrack_sync(x["eng"].handle))

    for f in range(a.warmup):
        step(f)
    sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(a.warmup, F):
        step(f)
    sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"streams": S, "engines": E, "calls_per_s": S * a.steps / dt,
                      "ms_per_step": 1000 * dt / a.steps,
                      "lib": os.environ.get("YTA_LIBRARY", "default")}), flush=True)


if __name__ == "__main__":
    main()
