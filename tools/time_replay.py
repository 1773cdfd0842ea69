"""Time the lapjv replay (lap_dense.hpp, one wave; yta_lap_padded KAT) on a GIoU-surge-shaped
cost matrix: more detections than trackers, every pair that does not overlap costs exactly 0 (the
reference's giou_batch gives non-overlapping pairs -1 -> 0 after the shift), a few overlapping
pairs per tracker cost -(iou-like) < 0.  Checks the assignment against oracle/lapjv.c and prints
both times.  GPU box: python tools/time_replay.py [--na 3874 --nb 1934]"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import lap as olap  # noqa: E402
from yolo_tracking_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--na", type=int, default=3874)
ap.add_argument("--nb", type=int, default=1934)
ap.add_argument("--per-col", type=int, default=4)
ap.add_argument("--seed", type=int, default=5)
args = ap.parse_args()
rng = np.random.default_rng(args.seed)
c = np.zeros((args.na, args.nb))
for j in range(args.nb):
    rows = rng.choice(args.na, size=args.per_col, replace=False)
    c[rows, j] = -rng.random(args.per_col) * 0.8 - 0.05
print(f"{args.na} x {args.nb}, {np.count_nonzero(c)} nonzero entries", flush=True)
t0 = time.perf_counter()
_, x_ref, _ = olap.lapjv(c, extend_cost=True)
t_cpu = time.perf_counter() - t0
x, _ = _lib.lap_padded(c)   # warm-up (module load, allocation)
t0 = time.perf_counter()
x, _ = _lib.lap_padded(c)
t_gpu = time.perf_counter() - t0
if os.environ.get("YTA_STAMPS_READ"):   # diagnostic library: phase split of the last solve
    import ctypes
    st = np.zeros(128, np.uint64)
    fn = _lib.load_library().yta_kat_debug_stamps
    fn.argtypes = [ctypes.c_void_p]
    _lib.check(fn(st.ctypes.data))
    print(f"phases 1-2 {(int(st[61]) - int(st[60])) / 100:.0f} us, phase 3 "
          f"{(int(st[62]) - int(st[61])) / 100:.0f} us (100 MHz stamps); sweeps {int(st[63])} "
          f"({int(st[64]) / 100:.0f} us incl. swaps), gathers {int(st[65])}, swap-to-front "
          f"{int(st[66]) / 100:.0f} us moving {int(st[67])} marked columns); sparse sweeps "
          f"{int(st[68])} ({int(st[69]) / 100:.0f} us, wave 0)", flush=True)
    if st[20] and st[21] and st[22]:
        print(f"  phase 1 column reduction {(int(st[20]) - int(st[60])) / 100:.0f} us, reduction "
              f"transfer {(int(st[21]) - int(st[20])) / 100:.0f} us, phase 2 "
              f"{(int(st[22]) - int(st[21])) / 100:.0f} us", flush=True)
same = np.array_equal(np.where(np.asarray(x) < args.nb, x, -1), np.where(x_ref < args.nb, x_ref, -1))
print(f"replay {t_gpu * 1e3:.1f} ms on the device, oracle/lapjv.c {t_cpu * 1e3:.1f} ms on one core, "
      f"assignments equal: {same}", flush=True)
sys.exit(0 if same else 1)
