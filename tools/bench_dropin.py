"""Drop-in latency: one stream through the reference's plugin surface, exactly as
examples/track.py drives it — `create_tracker(...)` then `tracker.update(dets, img)` with NumPy
in and out every frame (wall clock incl. host->device dets, kernels and
device->host outputs; median over frames 2..F after a warm-up frame).  Prints one JSON line per
tracker.

    python tools/bench_dropin.py [--trackers bytetrack,ocsort] [--frames 60]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SIZES = {"bytetrack": 1024, "ocsort": 256}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trackers", default="bytetrack,ocsort")
    ap.add_argument("--frames", type=int, default=60)
    a = ap.parse_args()
    from yolo_tracking_amd import create_tracker, get_tracker_config
    from yolo_tracking_amd.synth import make_frames
    for name in a.trackers.split(","):
        n = SIZES[name]
        kw = {} if name == "bytetrack" else {"low_conf_frac": 0.0}
        frames = [d for d, _ in make_frames(n, a.frames, seed=3, **kw)]
        C = int(64 * np.sqrt(n))
        img = np.zeros((C, C, 3), np.uint8)
        t = create_tracker(name, get_tracker_config(name), None, "cuda:0", False, False)
        dt = []
        for f, dets in enumerate(frames):
            d32 = dets.astype(np.float32)            # ultralytics hands float32 boxes
            t0 = time.perf_counter()
            out = t.update(d32, img)
            dt.append(time.perf_counter() - t0)
        med = float(np.median(dt[2:]))
        print(json.dumps({"tracker": name, "tracks_x_dets": f"{n}x{n}", "median_ms": 1e3 * med,
                          "calls_per_s": 1.0 / med, "frames": len(frames),
                          "rows_last_frame": int(np.asarray(out).reshape(-1, 8).shape[0]) if len(out) else 0}))


if __name__ == "__main__":
    main()
