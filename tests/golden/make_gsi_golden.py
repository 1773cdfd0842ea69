#!/usr/bin/env python3
"""Generate the GSI golden vectors from the reference (container-only; needs /root/reference).

    python tests/golden/make_gsi_golden.py        # writes tests/golden/gsi_mot17.npz

Inputs are MOT-format result rows built from the committed G1 ByteTrack outputs
(bytetrack_mot17.npz) the way examples/utils.py:8-28 writes them (frame_idx + 1, id, ltwh, conf,
cls, -1, every value through np.savetxt's '%d'), then read back as boxmot/postprocessing/gsi.py:66
does (np.loadtxt dtype=int).  The reference's own functions are then run on them:
  li_<seq>    linear_interpolation(rows, 20)            (gsi.py:12-30), float64 as returned
  gs_<seq>    gaussian_smooth(li, 10) as an array       (gsi.py:33-59), before the '%d' write
  out_<seq>   the file gsi() writes back, read as ints  (gsi.py:62-72)
plus a synthetic case with long gaps, single-row tracks and a track longer than tau**3 rows.
"""
import contextlib
import io
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import refshim  # noqa: E402

refshim.load()
from boxmot.postprocessing import gsi as ref_gsi  # noqa: E402

SEQS = ["MOT17_02_FRCNN", "MOT17_05_FRCNN", "MOT17_09_FRCNN"]


def mot_rows(g, seq):
    counts = g[seq + "__out_counts"]
    box = g[seq + "__out_box"]
    ints = g[seq + "__out_int"]
    score = g[seq + "__out_score"]
    frame = np.repeat(np.arange(1, len(counts) + 1), counts)
    x1, y1, x2, y2 = box.T
    mot = np.stack([frame, ints[:, 0], x1, y1, x2 - x1, y2 - y1, score, ints[:, 1],
                    -np.ones(len(frame))], axis=1)
    buf = io.StringIO()
    np.savetxt(buf, mot, fmt="%d")
    return np.loadtxt(io.StringIO(buf.getvalue()), dtype=int, delimiter=" ")


def synth_rows(seed=11):
    rng = np.random.default_rng(seed)
    rows = []
    for tid in range(1, 40):
        n_frames = int(rng.choice([1, 2, 5, 30, 120, 400, 1300])) if tid > 1 else 1300
        start = int(rng.integers(1, 50))
        frames = np.arange(start, start + n_frames)
        keep = rng.random(n_frames) > 0.25            # gaps of every length, some > interval
        keep[0] = True
        frames = frames[keep]
        x = 500 + np.cumsum(rng.normal(0, 3, len(frames)))
        y = 300 + np.cumsum(rng.normal(0, 3, len(frames)))
        w = 40 + rng.normal(0, 2, len(frames))
        h = 90 + rng.normal(0, 2, len(frames))
        for k, f in enumerate(frames):
            rows.append([f, tid, x[k], y[k], w[k], h[k], 0, 0, -1])
    rows = np.array(rows)
    rows = rows[rng.permutation(len(rows))]
    buf = io.StringIO()
    np.savetxt(buf, rows, fmt="%d")
    return np.loadtxt(io.StringIO(buf.getvalue()), dtype=int, delimiter=" ")


def run_case(name, rows, out):
    with contextlib.redirect_stdout(io.StringIO()):        # gsi.py:35,39 print the arrays
        li = ref_gsi.linear_interpolation(rows, 20)
        gs = np.asarray(ref_gsi.gaussian_smooth(li, 10), dtype=np.float64)
        with tempfile.TemporaryDirectory() as d:
            from pathlib import Path
            p = Path(d) / f"{name}.txt"
            np.savetxt(p, rows, fmt="%d")
            ref_gsi.gsi(mot_results_folder=Path(d), interval=20, tau=10)
            final = np.loadtxt(p, dtype=int, delimiter=" ")
    out[f"in_{name}"] = rows.astype(np.int64)
    out[f"li_{name}"] = np.asarray(li, dtype=np.float64)
    out[f"gs_{name}"] = gs
    out[f"out_{name}"] = final.astype(np.int64)
    print(f"{name}: {len(rows)} rows -> {len(li)} interpolated -> {len(final)} written")


def main():
    g = np.load(os.path.join(HERE, "bytetrack_mot17.npz"))
    out = {}
    for seq in SEQS:
        run_case(seq.replace("_", "-"), mot_rows(g, seq), out)
    run_case("MOT99-11-FRCNN", synth_rows(), out)   # synthetic (the name must match gsi.py:63)
    np.savez_compressed(os.path.join(HERE, "gsi_mot17.npz"), **out)
    print("wrote", os.path.join(HERE, "gsi_mot17.npz"))


if __name__ == "__main__":
    main()
