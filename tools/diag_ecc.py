"""ECC phase timeline (GPU box, diagnostic library): YTA_LIBRARY=tools/variants/libyta_eccst.so
python tools/diag_ecc.py [--streams S] [--mode M] -> block 0's microseconds per phase of k_ecc,
summed over its Gauss-Newton iterations, for one frame pair of the CMC bench scene."""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from bench_cmc import frames_for  # noqa: E402
from yolo_tracking_amd import _lib  # noqa: E402
from yolo_tracking_amd.motion.ecc import EccEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--streams", type=int, default=1)
ap.add_argument("--mode", type=int, default=1)
args = ap.parse_args()
fr = frames_for(args.streams, 3, 1080, 1920, 3)
eng = EccEngine(args.streams, args.mode, 1e-5, 100, 0.1, 0, 1080, 1920)
fn = eng.lib.yta_ecc_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
names = ["setup", "tables", "pass A", "block sums", "pass B", "solves", "pass C"]
for f in range(3):
    eng.apply(list(fr[f]))
    st = np.zeros(9, np.uint64)
    _lib.check(fn(eng.handle, st.ctypes.data))
    it = int(st[7])
    tot = float(st[:7].sum()) / 100.0
    print(f"frame {f}: {it} iterations, {tot:.1f} us:",
          ", ".join(f"{n} {float(st[i]) / 100.0:.1f}" for i, n in enumerate(names)),
          f"| shader clock {float(st[8]) / max(tot, 1e-9):.0f} MHz")
