#!/usr/bin/env python3
"""CPU check of tools/lapjv_sparse_proto.c against oracle/lapjv.c: the same x, y and column prices
(bit for bit) on GIoU-surge-shaped matrices (every non-overlapping pair exactly 0, a few negative
entries per tracker column; zero-padded to square as extend_cost does) and on denser / positive
ones; prints how many phase-3 sweeps stayed sparse and both solve times.

    python tools/lapjv_sparse_check.py [--quick]
"""
import argparse
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "lapjv_sparse_proto.c")
OUT = os.path.join(REPO, "tools", "liblapjv_sparse_proto.so")


def load():
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", SRC, "-o", OUT])
    proto = ctypes.CDLL(OUT)
    orc = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    for f in (proto.proto_lapjv_square,):
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_void_p, ctypes.c_void_p]
    orc.oracle_lapjv_square.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]
    return proto, orc


def surge(rng, na, nb, per_col, pos_frac=0.0):
    c = np.zeros((na, nb))
    for j in range(nb):
        rows = rng.choice(na, size=per_col, replace=False)
        c[rows, j] = -rng.random(per_col) * 0.8 - 0.05
    if pos_frac:
        m = rng.random((na, nb)) < pos_frac
        c[m] = rng.random(int(m.sum())) * 0.3
    n = max(na, nb)
    sq = np.zeros((n, n))
    sq[:na, :nb] = c
    return sq


def run(proto, orc, sq):
    n = len(sq)
    sq = np.ascontiguousarray(sq)
    x0, y0 = np.empty(n, np.int32), np.empty(n, np.int32)
    t0 = time.perf_counter()
    assert orc.oracle_lapjv_square(n, sq.ctypes.data, x0.ctypes.data, y0.ctypes.data) == 0
    t_o = time.perf_counter() - t0
    x1, y1 = np.empty(n, np.int32), np.empty(n, np.int32)
    v1 = np.empty(n)
    st = np.zeros(3, np.int64)
    t0 = time.perf_counter()
    proto.proto_lapjv_square(n, sq.ctypes.data, x1.ctypes.data, y1.ctypes.data, v1.ctypes.data,
                             st.ctypes.data)
    t_p = time.perf_counter() - t0
    return np.array_equal(x0, x1) and np.array_equal(y0, y1), st, t_o, t_p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    proto, orc = load()
    cases = [(200, 100, 4, 0.0), (100, 200, 3, 0.0), (600, 300, 4, 0.0), (300, 300, 6, 0.0),
             (500, 250, 4, 0.01), (400, 200, 2, 0.2)]
    if not args.quick:
        cases += [(2000, 1000, 4, 0.0), (3874, 1934, 4, 0.0)]
    ok_all = True
    for seed in range(3 if args.quick else 2):
        for na, nb, pc, pf in cases:
            rng = np.random.default_rng(seed * 1000 + na + nb)
            ok, st, t_o, t_p = run(proto, orc, surge(rng, na, nb, pc, pf))
            ok_all &= ok
            print(f"{na}x{nb} per_col {pc} pos {pf}: equal {ok}  sweeps sparse {st[0]} dense "
                  f"{st[1]} gathers {st[2]}  oracle {t_o * 1e3:.1f} ms  proto {t_p * 1e3:.1f} ms",
                  flush=True)
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
