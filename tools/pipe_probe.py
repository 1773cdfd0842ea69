#!/usr/bin/env python3
"""Probe of the pipelined host-buffer path (yta_bytetrack_submit / _collect) in a fresh process.

    python tools/pipe_probe.py [--streams 2048] [--first 10] [--frames 8] [--extra-streams K]

Runs bench.py's synchronous and pipelined PCIe legs on the same synthetic frames and prints one
JSON line per leg with the library's accounting (yta_bytetrack_pipe_stats: direct vs staged
bytes each way, host time in submit / collect, GPU time of each frame's copy-in, kernels and
copy-out, and the frame's whole span).  --extra-streams creates K HIP streams first (as the
headline engines and torch do inside bench.py) to see whether the copy / compute streams' queue
placement matters.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def host_allocator(kind):
    """Page-locked numpy arrays from the HIP runtime torch loaded (hipHostMalloc, or mmap'd memory
    registered with hipHostRegister); never freed (probe process)."""
    import ctypes
    import glob
    import mmap

    import torch
    lib = ctypes.CDLL(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib",
                                             "libamdhip64.so*"))[0])
    keep = []

    def alloc(shape, dtype):
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        if kind == "hiphostmalloc":
            p = ctypes.c_void_p()
            assert lib.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), 0) == 0
            buf = (ctypes.c_char * n).from_address(p.value)
        else:
            m = mmap.mmap(-1, n)
            buf = (ctypes.c_char * n).from_buffer(m)
            keep.append(m)
            assert lib.hipHostRegister(ctypes.c_void_p(ctypes.addressof(buf)), ctypes.c_size_t(n),
                                       0) == 0
        keep.append(buf)
        return np.frombuffer(buf, dtype=dtype).reshape(shape)
    return alloc


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--streams", type=int, default=2048)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--first", type=int, default=10)
    p.add_argument("--frames", type=int, default=8)
    p.add_argument("--extra-streams", type=int, default=0)
    p.add_argument("--cap-mult", type=int, default=3, help="pipelined engine capacity, x N")
    p.add_argument("--legs", default="sync,sync_pinned,pipe,pipe_pinned,pipe_pinned_f32")
    p.add_argument("--alloc", default="torch", choices=["torch", "hiphostmalloc", "register"],
                   help="page-locked caller buffers: torch's pinned allocator, hipHostMalloc, or "
                        "page-aligned numpy memory registered with hipHostRegister")
    a = p.parse_args()
    import torch

    import bench
    from yolo_tracking_amd.synth import SyntheticStream
    torch.cuda.set_device(0)
    if a.alloc != "torch":
        bench.pinned_empty = host_allocator(a.alloc)
    S, N = a.streams, a.n
    gens = [SyntheticStream(N, bench.stream_seeds(1000, 0, S)[s]) for s in range(S)]
    t0 = time.time()
    frames = []
    for _ in range(a.first + a.frames):
        fr = np.empty((S * N, 6))
        for s, g in enumerate(gens):
            fr[s * N:(s + 1) * N] = g.next_frame()[0]
        frames.append(fr)
    gen_s = time.time() - t0
    extra = [torch.cuda.Stream() for _ in range(a.extra_streams)]

    def frame_of(f):
        return frames[f]
    env = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "HSA_ENABLE_SDMA",
                                          "HIP_FORCE_DEV_KERNARG", "OMP_NUM_THREADS")}
    print(json.dumps({"probe": "env", "env": env, "alloc": a.alloc, "gen_s": round(gen_s, 1),
                      "extra_streams": len(extra)}), flush=True)
    for leg in a.legs.split(","):
        t = time.time()
        if leg == "sync":
            r = bench.pcie_inclusive(frame_of, S, N, 0, first=a.first, frames=a.frames)
        elif leg == "sync_pinned":
            r = bench.pcie_inclusive(frame_of, S, N, 0, first=a.first, frames=a.frames, pinned=True)
        elif leg == "pipe":
            r = bench.pcie_pipelined(frame_of, S, N, 0, first=a.first, frames=a.frames,
                                     cap_mult=a.cap_mult)
        elif leg == "pipe_pinned":
            r = bench.pcie_pipelined(frame_of, S, N, 0, first=a.first, frames=a.frames,
                                     pinned=True, cap_mult=a.cap_mult)
        elif leg == "pipe_pinned_f32":
            r = bench.pcie_pipelined(frame_of, S, N, 0, first=a.first, frames=a.frames,
                                     pinned=True, f32=True, cap_mult=a.cap_mult)
        else:
            raise SystemExit(f"unknown leg {leg}")
        r.pop("note", None)
        print(json.dumps({"probe": leg, "wall_s": round(time.time() - t, 1), **r}), flush=True)


if __name__ == "__main__":
    main()
