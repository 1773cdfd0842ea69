#!/usr/bin/env python3
"""GPU box: PCIe copy rates of the host-buffer path's transfer sizes (100 MB of detections in,
134 MB of rows out per 2048-stream step): host->device alone, device->host alone, and both at
once on two streams (pinned buffers), to see what bounds the pipelined host path."""
import json
import time

import torch

H2D, D2H, REP = 100663296, 134217728, 10
hin = torch.empty(H2D, dtype=torch.uint8, pin_memory=True)
hout = torch.empty(D2H, dtype=torch.uint8, pin_memory=True)
din = torch.empty(H2D, dtype=torch.uint8, device="cuda")
dout = torch.empty(D2H, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REP):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / REP


def h2d():
    with torch.cuda.stream(s1):
        din.copy_(hin, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        hout.copy_(dout, non_blocking=True)


def both():
    h2d()
    d2h()


timed(both)
a, b, c = timed(h2d), timed(d2h), timed(both)
print(json.dumps({"h2d_ms": a * 1e3, "h2d_gbs": H2D / a / 1e9, "d2h_ms": b * 1e3,
                  "d2h_gbs": D2H / b / 1e9, "both_ms": c * 1e3,
                  "both_gbs": (H2D + D2H) / c / 1e9}))
