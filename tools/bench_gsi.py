#!/usr/bin/env python3
"""GSI post-processing (boxmot/postprocessing/gsi.py) on the MI355X vs the CPU oracle.

    python tools/bench_gsi.py [--ids 400] [--frames 900] [--reps 3]

Tables: the four golden MOT tables (tests/golden/gsi_mot17.npz) and one synthetic MOT20-sized
table (ids x frames, 20 % of rows dropped).  Per table: rows in / out, end-to-end wall time of
linear_interpolation + gaussian_smooth through the C ABI (host buffers in and out, as gsi() uses
it), the oracle's time (NumPy / SciPy, one thread), the largest |GPU - oracle| prediction and the
Cholesky work (sum over tracks of n * w^2, band width w).  One JSON line per table.
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import yolo_tracking_amd.postprocessing.gsi as pg  # noqa: E402
from oracle import gsi as og  # noqa: E402


def synth(ids, frames, seed=5):
    rng = np.random.default_rng(seed)
    rows = []
    for tid in range(1, ids + 1):
        n = int(rng.integers(20, frames))
        start = int(rng.integers(1, frames - n + 2))
        f = np.arange(start, start + n)
        f = f[rng.random(n) > 0.2]
        x = 900 + np.cumsum(rng.normal(0, 3, len(f)))
        y = 500 + np.cumsum(rng.normal(0, 3, len(f)))
        rows.append(np.stack([f, np.full(len(f), tid), x, y, np.full(len(f), 40.0),
                              np.full(len(f), 100.0), np.ones(len(f)), np.zeros(len(f)),
                              -np.ones(len(f))], 1))
    return np.round(np.concatenate(rows)).astype(int)


def work(li, tau):
    tot = 0
    for id_ in set(li[:, 1]):
        t = li[li[:, 1] == id_][:, 0].astype(np.float64)
        w = pg._band_width(t, float(og.length_scale_of(len(t), tau)))
        tot += len(t) * (w + 1) ** 2
    return tot


def run(name, tab, reps, cpu=True):
    pg.gaussian_smooth(pg.linear_interpolation(tab[:50], 20), 10)          # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        li = pg.linear_interpolation(tab, 20)
        gs = pg.gaussian_smooth(li, 10)
        ts.append(time.perf_counter() - t0)
    rec = {"table": name, "rows_in": int(len(tab)), "rows_out": int(len(li)),
           "tracks": int(len(set(li[:, 1]))), "gpu_s": min(ts), "chol_work": int(work(li, 10))}
    if cpu:
        t0 = time.perf_counter()
        lo = og.linear_interpolation(tab, 20)
        go = og.gaussian_smooth(lo, 10)
        rec["cpu_oracle_s"] = time.perf_counter() - t0
        rec["cpu_cores"] = 1
        rec["speedup"] = rec["cpu_oracle_s"] / rec["gpu_s"]
        assert np.array_equal(li, lo)
        rec["max_abs_err_px"] = float(np.abs(np.asarray(gs)[:, 2:6] - np.asarray(go)[:, 2:6]).max())
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ids", type=int, default=400)
    ap.add_argument("--frames", type=int, default=900)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    g = np.load(os.path.join(REPO, "tests", "golden", "gsi_mot17.npz"))
    for n in sorted({k.split("_", 1)[1] for k in g.files}):
        run(n, g["in_" + n], a.reps)
    run(f"synthetic {a.ids} ids x {a.frames} frames", synth(a.ids, a.frames), a.reps)


if __name__ == "__main__":
    main()
