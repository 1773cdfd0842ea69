#!/usr/bin/env python3
"""Design experiment (CPU): how many rows of the OCSORT-family first-round solve are left for
Dijkstra after the claims of lap_rect.hpp, and after rounds of parallel (Jacobi) augmenting row
reduction on top of them, on the first-round cost matrices of the C5 synthetic workload (captured
from oracle/hybridsort.py's associate_reid).

    python tools/sim_arr.py [N] [FRAMES] [ROUNDS]

Checks that the final assignment is optimal (equal cost to scipy's linear_sum_assignment) when
every row is assigned by the rounds alone.
"""
import os
import sys

import numpy as np
from scipy.optimize import linear_sum_assignment

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle.hybridsort as H  # noqa: E402
from yolo_tracking_amd.synth import make_frames  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
NF = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ROUNDS = int(sys.argv[3]) if len(sys.argv) > 3 else 12
captured = []
STATS = [None] if os.environ.get('ARR_STATS') else []
_orig = H.linear_assignment_padded


def _cap(c):
    if not captured or captured[-1][0] != len(frames_done):
        captured.append((len(frames_done), np.array(c)))
    return _orig(c)


H.linear_assignment_padded = _cap
frames_done = []


def claims(c):
    u = c.min(1)
    j1 = c.argmin(1)
    s = np.sort(c, 1)
    s2 = s[:, 1] - s[:, 0]
    return u, j1, s2


def jacobi_arr(c, rounds, rule="delta"):
    """Parallel ARR: v (column prices, decreasing), owner, assignment; returns free counts."""
    n, m = c.shape
    v = np.zeros(m)
    x = -np.ones(n, int)
    y = -np.ones(m, int)
    free = np.arange(n)
    counts = [n]
    for r in range(rounds):
        if len(free) == 0:
            break
        red = c[free] - v[None, :]
        j1 = red.argmin(1)
        u1 = red[np.arange(len(free)), j1]
        red2 = red.copy()
        red2[np.arange(len(free)), j1] = np.inf
        j2 = red2.argmin(1)
        u2 = red2[np.arange(len(free)), j2]
        d = u2 - u1
        # tie (d == 0) on an owned j1: take j2 instead when j2 is free (tight there too)
        alt = (d == 0) & (y[j1] >= 0) & (y[j2] < 0)
        tgt = np.where(alt, j2, j1)
        dd = np.where(alt, 0.0, d)
        # winner per column: largest decrement, lowest row on ties
        order = np.lexsort((free, -dd, tgt))
        first = np.ones(len(order), bool)
        first[1:] = tgt[order][1:] != tgt[order][:-1]
        win = order[first]
        newfree = list(free[np.setdiff1d(np.arange(len(free)), win)])
        for w in win:
            i, j = free[w], tgt[w]
            v[j] -= dd[w]
            if y[j] >= 0:
                x[y[j]] = -1
                newfree.append(y[j])
            y[j] = i
            x[i] = j
        free = np.array(sorted(newfree), int)
        counts.append(len(free))
        if STATS:
            STATS.append((len(free), int((dd == 0).sum()), len(np.unique(tgt)), int(alt.sum())))
    # feasibility / tightness check: u_i = c_i,x_i - v_x_i must equal min_j (c_ij - v_j)
    asg = x >= 0
    red = c - v[None, :]
    ok = np.allclose(red[asg].min(1), red[np.nonzero(asg)[0], x[asg]], rtol=0, atol=1e-9)
    return counts, x, ok


tr = H.HybridSortOracle(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
                        asso_func="giou", inertia=0.2)
for f, (dets, feats) in enumerate(make_frames(N, NF, 2000, emb_dim=512, low_conf_frac=0.0)):
    frames_done.append(f)
    tr.update(dets, feats / np.linalg.norm(feats))
    if not captured or captured[-1][0] != len(frames_done):
        continue
    c = captured[-1][1]
    n, m = c.shape
    if os.environ.get("SAVE_DIR"):
        np.save(os.path.join(os.environ["SAVE_DIR"], f"c{N}_f{f}.npy"), c)
    if n > m:
        print(f"frame {f}: {n} x {m} (rows > cols: not the rectangular case)")
        continue
    u, j1, s2 = claims(c)
    owner = {}
    for i in range(n):
        owner.setdefault(j1[i], i)
    print(f"frame {f}: {n} x {m}, claims leave {n - len(owner)} free rows", flush=True)
    counts, x, ok = jacobi_arr(c, ROUNDS)
    msg = f"  jacobi ARR free rows per round {counts}, duals feasible+tight {ok}"
    if counts[-1] == 0:
        r, k = linear_sum_assignment(c)
        opt = c[r, k].sum()
        got = c[np.arange(n), x].sum()
        msg += f", cost {got:.12g} vs optimum {opt:.12g} (diff {got - opt:.3g})"
    print(msg, flush=True)
