#!/usr/bin/env python3
"""Design experiment (CPU) for the OCSORT-family first-round solve: rounds of speculative
shortest-augmenting-path searches from every free row at once, committed in row order while their
scanned column sets stay disjoint (a search whose columns no earlier commit of the round touched
sees exactly the duals and owners a sequential search would: the commits only lower the prices of
their own columns).  Prints, per matrix: the free rows after the claims, the rounds, the
per-round critical path (longest search, in row scans), the total row scans, and checks the
optimum against scipy.

    python tools/sim_lap_parallel.py MATRIX.npy [...]      (matrices saved by tools/sim_arr.py)
"""
import sys

import numpy as np
from scipy.optimize import linear_sum_assignment


def claims(c):
    n, m = c.shape
    u = c.min(1)
    j1 = c.argmin(1)
    srt = np.sort(c, 1)
    S2[:] = srt[:, 1] - srt[:, 0]
    x = -np.ones(n, int)
    y = -np.ones(m, int)
    for i in range(n):          # lowest row wins
        if y[j1[i]] < 0:
            y[j1[i]] = i
            x[i] = j1[i]
    return u.copy(), np.zeros(m), x, y


def search(c, r, u, v, y):
    """Dijkstra from free row r on reduced costs c - u - v (>= 0).  Returns (sink, pred, d,
    scanned list (in order), row scans)."""
    m = c.shape[1]
    d = c[r] - u[r] - v
    pred = np.full(m, r)
    done = np.zeros(m, bool)
    scanned = []
    scans = 1
    while True:
        dd = np.where(done, np.inf, d)
        j = int(np.argmin(dd))
        done[j] = True
        scanned.append(j)
        if y[j] < 0:
            return j, pred, d, scanned, scans
        i = y[j]
        nd = d[j] + c[i] - u[i] - v
        upd = (~done) & (nd < d)
        d = np.where(upd, nd, d)
        pred = np.where(upd, i, pred)
        scans += 1


def search_pruned(c, r, u, v, y, s2):
    """lap_rect.hpp's search: an owned column's row is relaxed only while d_j + s2[row] < B (B =
    the cheapest free column reached).  Returns (sink, pred, d, touched columns (d < B, + sink),
    row scans, new s2 values of the relaxed rows)."""
    m = c.shape[1]
    d = c[r] - u[r] - v
    pred = np.full(m, r)
    rel = np.zeros(m, bool)
    owned = y >= 0
    s2n = {}
    scans = 1
    xi = -1
    bprev = np.inf
    while True:
        fd = np.where(owned, np.inf, d)
        sink = int(np.argmin(fd))
        B = fd[sink]
        bound = np.where(owned, s2[np.maximum(y, 0)], 0.0)
        for i_, val in s2n.items():
            pass
        cand = owned & ~rel & (d + bound < bprev)
        cd = np.where(cand, d, np.inf)
        ja = int(np.argmin(cd))
        ma = cd[ja]
        if not ma < B:
            break
        rel[ja] = True
        i = y[ja]
        base = ma
        rc = c[i] - u[i] - v
        mo = np.min(np.where(np.arange(m) == ja, np.inf, rc))
        s2[i] = mo          # exact for the current duals (lap_rect.hpp: s2c of the row's column)
        nd = base + rc
        upd = (~rel) & (nd < d)
        d = np.where(upd, nd, d)
        pred = np.where(upd, i, pred)
        bprev = B
        scans += 1
    touched = [int(j) for j in np.nonzero(owned & (d < B))[0]] + [sink]
    return sink, pred, d, touched, scans


def commit(r, sink, pred, d, scanned, u, v, x, y, s2=None):
    B = d[sink]
    for j in scanned:
        if j != sink and y[j] >= 0 and d[j] < B:
            dl = B - d[j]
            u[y[j]] += dl
            v[j] -= dl
            if s2 is not None:
                s2[y[j]] -= dl
    u[r] += B
    j = sink
    while True:
        i = pred[j]
        y[j] = i
        nx = x[i]
        x[i] = j
        if s2 is not None:
            s2[i] = 0.0
        if i == r:
            break
        j = nx


def solve_parallel(c, pruned=False):
    u, v, x, y = claims(c)
    free = [i for i in range(c.shape[0]) if x[i] < 0]
    n0 = len(free)
    rounds, crit, total = 0, 0, 0
    while free:
        rounds += 1
        if pruned:
            snap = S2.copy()
            res = []
            for r in free:
                s2w = snap.copy()
                res.append((r,) + search_pruned(c, r, u, v, y, s2w) + (s2w,))
        else:
            res = [(r,) + search(c, r, u, v, y) + (None,) for r in free]
        crit += max(s[-2] for s in res)
        total += sum(s[-2] for s in res)
        touched = set()
        left = []
        for r, sink, pred, d, scanned, scans, s2w in res:
            S = set(scanned)
            if S & touched:
                left.append(r)
                continue
            touched |= S
            if s2w is not None:   # the relaxed rows' exact bounds (rows of the touched columns)
                rows = [y[j] for j in scanned if y[j] >= 0]
                S2[rows] = s2w[rows]
            commit(r, sink, pred, d, scanned, u, v, x, y, S2 if pruned else None)
        free = left
    return n0, rounds, crit, total, x


def solve_sequential(c, pruned=False):
    u, v, x, y = claims(c)
    free = [i for i in range(c.shape[0]) if x[i] < 0]
    total = 0
    for r in free:
        if pruned:
            sink, pred, d, scanned, scans = search_pruned(c, r, u, v, y, S2)
            commit(r, sink, pred, d, scanned, u, v, x, y, S2)
        else:
            sink, pred, d, scanned, scans = search(c, r, u, v, y)
            commit(r, sink, pred, d, scanned, u, v, x, y)
        total += scans
    return total, x


def arr_then_sap(c, rounds, rule=1):
    """Jacobi ARR rounds (round 1 = the row pre-pass's bids: largest decrement wins a column,
    lowest row on ties), then lap_rect.hpp's pruned searches for the rows still free."""
    n, m = c.shape
    srt = np.sort(c, 1)
    S2[:] = srt[:, 1] - srt[:, 0]
    u = c.min(1).copy()
    v = np.zeros(m)
    x = -np.ones(n, int)
    y = -np.ones(m, int)
    free = np.arange(n)
    counts = []
    scans_arr = 0
    for r in range(rounds):
        if len(free) == 0:
            break
        if r > 0:
            scans_arr += len(free)
        red = c[free] - v[None, :]
        j1 = red.argmin(1)
        u1 = red[np.arange(len(free)), j1]
        red[np.arange(len(free)), j1] = np.inf
        j2 = red.argmin(1)
        u2 = red[np.arange(len(free)), j2]
        d = u2 - u1
        alt = (d == 0) & (y[j1] >= 0) & (y[j2] < 0)
        tgt = np.where(alt, j2, j1)
        dd = np.where(alt, 0.0, d)
        order = np.lexsort((free, -dd, tgt))
        first = np.ones(len(order), bool)
        first[1:] = tgt[order][1:] != tgt[order][:-1]
        win = order[first]
        isw = np.zeros(len(free), bool)
        isw[win] = True
        u[free] = u1                      # losers: their row minimum under the current prices
        newfree = list(free[~isw])
        # bidders per column and the runner-up decrement
        so = order
        cnt = np.bincount(tgt, minlength=m)
        second = np.zeros(m)
        for k in range(len(so)):
            if not first[k] and (k == 0 or first[k - 1]):
                second[tgt[so[k]]] = dd[so[k]]
        for w in win:
            i, j = free[w], tgt[w]
            contested = cnt[j] > 1 or y[j] >= 0
            if rule == 1 or (rule == 2 and contested):
                dec = dd[w]
            elif rule == 3 and contested:
                dec = second[j] if (cnt[j] > 1 and y[j] < 0) else dd[w]
            else:
                dec = 0.0
            v[j] -= dec
            if y[j] >= 0:
                x[y[j]] = -1
                newfree.append(y[j])
            y[j] = i
            x[i] = j
            u[i] = c[i, j] - v[j]
            S2[i] = (u2[w] - u1[w] - dec) if not alt[w] else 0.0
        free = np.array(sorted(newfree), int)
        counts.append(len(free))
    total = 0
    for r in free:
        sink, pred, d, scanned, scans = search_pruned(c, r, u, v, y, S2)
        commit(r, sink, pred, d, scanned, u, v, x, y, S2)
        total += scans
    return counts, scans_arr, total, x


S2 = None
PRUNED = True
if sys.argv[1] == "arr":
    for p in sys.argv[3:]:
        c = np.load(p)
        n = c.shape[0]
        S2 = np.zeros(n)
        seq, xs = solve_sequential(c, True)
        r, k = linear_sum_assignment(c)
        opt = c[r, k].sum()
        line = f"{p}: seq scans {seq}"
        for R in [int(q) for q in sys.argv[2].split(",")]:
            for rule in (1,):
                counts, sa, tot, x = arr_then_sap(c, R, rule)
                line += f" | R{R}v{rule} free {counts} arr {sa} sap {tot} diff {c[np.arange(n), x].sum() - opt:.2g}"
        print(line, flush=True)
    sys.exit(0)
for p in sys.argv[1:]:
    c = np.load(p)
    n = c.shape[0]
    S2 = np.zeros(n)
    seq, xs = solve_sequential(c, PRUNED)
    n0, rounds, crit, total, x = solve_parallel(c, PRUNED)
    r, k = linear_sum_assignment(c)
    opt = c[r, k].sum()
    print(f"{p}: {c.shape[0]}x{c.shape[1]} free after claims {n0}; sequential scans {seq}; "
          f"parallel rounds {rounds}, critical path {crit} scans, total {total}; "
          f"cost diff seq {c[np.arange(n), xs].sum() - opt:.3g} par {c[np.arange(n), x].sum() - opt:.3g}",
          flush=True)
