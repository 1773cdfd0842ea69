#!/usr/bin/env python3
"""Throughput of the MI355X ByteTrack update() (BASELINE.json headline metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--streams S] [--n 1024]

A step = one `tracker.update()` frame for every one of the S independent streams on each GPU
(each stream: 1024 tracks x 1024 detections per frame, SURVEY.md §8(d) synthetic generator).
All frames are staged in HBM before the timed region; the engine's device-buffer entry point
runs the whole update on the GPU (outputs stay in HBM).  N > 1: one process per GPU
(torch.distributed.run), streams sharded per rank, no data-path collective, barrier + max over
ranks around the timed region (scaling "weak": per-GPU work is fixed).

Rank 0 prints one JSON line with `roofline` (dominant kernel, HIP events on the engine stream)
and `cpu_baseline` (the oracle's CPU restatement on this host, 1 core, bounded sample).
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PHASES = ["s1_prep", "s1_edges", "s1_lap", "stage23", "apply", "finish"]
STATS = ["dets", "high", "second", "pool", "act", "unc", "left", "rest", "births", "t2", "l2",
         "tracked", "lost", "out", "edges1", "edges23", "fallback1", "fallback23", "lazy", "res1"]
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Canonical algorithmic bytes per update: ByteTrack 1024 x 1024
BYTES_PER_UPDATE_1024 = 19_259_392


def algorithmic_bytes(n, m):
    """B = 4*S*N + 56*M + 16*N*M + 64*N with S = 576 (ByteTrack)."""
    return 4 * 576 * n + 56 * m + 16 * n * m + 64 * n


def kernel_bytes(phase, st):
    """Algorithmic HBM bytes one launch of `phase` must move, from the last frame's counts summed
    over streams.  Kalman record = 24 f64 (192 B), track meta = 48 B, box = 32 B,
    detection row = 48 B, candidate edge = 12 B (int column + f64 cost)."""
    pool, unc, high, dets = st["pool"], st["unc"], st["high"], st["dets"]
    act, lazy = st["act"], st["lazy"]
    lost_list = pool - act
    matched = st["tracked"]            # tracks updated this frame (upper bound: tracked list)
    if phase == "s1_prep":
        # dets read, measurement / conf / cls written; high and low lists with boxes (+ score);
        # tracked list, flags and Kalman mean of every pool / unconfirmed track (+ the lazy frame
        # of lost ones), pool / unconfirmed lists with boxes written
        return (dets * (48 + 48) + high * (4 + 32 + 8) + st["second"] * (4 + 32)
                + (act + unc) * (4 + 4 + 64 + 4 + 32) + lost_list * (4 + 4 + 4 + 64 + 4 + 32))
    if phase == "s1_edges":
        # high boxes + scores read once (grid built in LDS), every pool box read, edge count and
        # edges written, single-edge matches: x1 of every pool row, y1 of every high detection
        return high * (32 + 8 + 4) + pool * (32 + 4 + 4) + st["edges1"] * 12
    if phase == "s1_lap":
        # edge counts and the edges left after the single-edge components read, the solver's
        # matches written
        return pool * 4 + st["res1"] * (12 + 8)
    if phase == "apply":
        # every pool / unconfirmed track but the lazily predicted lost ones: Kalman record + meta
        # read, record written; matched tracks: meta written, the detection's row read; every
        # pool item: index + stage results read, stage-1 kind written
        touched = pool - lazy + unc
        return touched * (192 + 48 + 192) + matched * (48 + 48) + pool * (4 + 4 + 4 + 4) + unc * 8
    if phase == "stage23":
        return (pool * (4 + 48 + 4) + high * (4 + 8 + 8) + st["left"] * (8 + 32 + 4)
                + st["second"] * (32 + 4) + unc * (32 + 4) + st["rest"] * (4 + 32 + 8 + 4))
    if phase == "finish":
        # lost list expiry (slot, flags, lost frame); tracked' boxes (mean), lost' means (lazily
        # predicted) for duplicate removal, list entries; output rows: mean + meta read, row
        # written; births: record + meta written
        return (lost_list * 12 + st["t2"] * (32 + 12) + st["l2"] * (64 + 4 + 12)
                + st["out"] * (32 + 48 + 64) + st["births"] * (192 + 48))
    return 0


def pmc_traffic(streams, n, queues):
    """HBM bytes per launch of the roofline kernel, and per step of the whole frame (every kernel
    of every engine), from the committed rocprofv3 PMC summary (profiles/roofline_traffic.json,
    FETCH_SIZE x 2 + WRITE_SIZE in separate passes), when it was measured on this same workload;
    else None."""
    f = os.path.join(REPO, "profiles", "roofline_traffic.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None, None, None
    if d.get("streams") == streams and d.get("n") == n and d.get("queues", 1) == queues:
        return d["hbm_bytes_per_launch"], d.get("hbm_bytes_per_step"), d.get("tag")
    return None, None, None


# ---------------------------------------------------------------- multi-rank harness (N > 1)
def stream_seeds(seed, rank, streams):
    """Rank r owns streams [r*S, (r+1)*S): disjoint seeds, so ranks shard the job (weak scaling)."""
    return [seed + rank * streams + s for s in range(streams)]


def timed_region(run_steps, sync, dist):
    """Barrier + device sync on both sides of the timed region; returns this rank's seconds."""
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run_steps()
    sync()
    if dist:
        dist.barrier()
    sync()
    return time.perf_counter() - t0


def max_over_ranks(elapsed, dist, device):
    """The job's time is the slowest rank's (all_reduce MAX; RCCL on the GPU box, gloo in tests)."""
    if not dist:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(world, streams, steps, elapsed):
    """Whole-job update calls per second over all ranks."""
    return world * streams * steps / elapsed


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--streams", type=int, default=2048, help="streams per GPU")
    p.add_argument("--n", type=int, default=1024, help="tracks = detections per frame")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe) leg")
    p.add_argument("--no-isolated", action="store_true",
                   help="skip the engine-0-alone frames after the timed region (profiling runs)")
    p.add_argument("--cpu-frames", type=int, default=40)
    p.add_argument("--seed", type=int, default=1000)
    p.add_argument("--queues", type=int, default=2,
                   help="engines per GPU, each on its own HIP stream, streams split between them")
    return p.parse_args()


def gen_stream_frames(n, frames, seed):
    from yolo_tracking_amd.synth import make_frames
    return [d for d, _ in make_frames(n, frames, seed)]


def cpu_baseline(n, frames, seed):
    """Time the oracle (CPU restatement: NumPy ByteTrack + C lapjv) on one stream, 1 thread."""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    code = (
        "import sys,time,json; sys.path.insert(0,%r)\n"
        "from oracle.bytetrack import ByteTrackOracle\n"
        "from yolo_tracking_amd.synth import make_frames\n"
        "fr=[d for d,_ in make_frames(%d,%d,%d)]\n"
        "t=ByteTrackOracle(0.5,0.8,30,30); t.update(fr[0])\n"
        "t0=time.perf_counter()\n"
        "for d in fr[1:]: t.update(d)\n"
        "dt=time.perf_counter()-t0\n"
        "print(json.dumps({'frames':len(fr)-1,'seconds':dt}))\n" % (REPO, n, frames, seed))
    try:
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           timeout=900)
        res = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as exc:  # report, never fail the bench on the baseline leg
        return {"value": None, "unit": "calls/s", "cores": 1, "kind": "port",
                "sample": f"failed: {exc}"}
    return {"value": res["frames"] / res["seconds"], "unit": "calls/s", "cores": 1, "kind": "port",
            "sample": f"oracle ByteTrack (NumPy + C lapjv), 1 stream {n}x{n}, frames 2..{frames} "
                      f"of seed {seed}, {res['seconds']:.1f} s, 1 thread"}


def pcie_inclusive(host, off, S, N, device, frames=8):
    """The same workload through the host-buffer ABI (yta_bytetrack_update: packed host dets in,
    output rows back to the host every call, synchronous), on a fresh engine: rank 0's report
    of the PCIe-inclusive rate.  Never `value`."""
    from yolo_tracking_amd import ByteTrackEngine, _lib
    # capacity 3N: the host path reserves ahead of need (tracked + lost + this frame's dets,
    # ~2.2N in the steady state) and would otherwise regrow the engine on the first frames
    eng = ByteTrackEngine(S, track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30,
                          device=device, track_capacity=3 * N, max_dets=N)
    lib, h = eng.lib, eng.handle
    out = np.empty((S * N, 8))   # <= one row per detection
    out_off = np.zeros(S + 1, np.int32)
    nid = np.zeros(S, np.int64)
    frames = min(frames, len(host))
    dets = [np.ascontiguousarray(host[f]) for f in range(frames)]
    offs = [np.ascontiguousarray(off[f]) for f in range(frames)]

    def call(f):
        _lib.check(lib.yta_bytetrack_update(h, dets[f].ctypes.data, offs[f].ctypes.data,
                                            nid.ctypes.data, out.ctypes.data, len(out),
                                            out_off.ctypes.data))
    call(0)
    call(1)
    dts = []
    for f in range(2, frames):
        t0 = time.perf_counter()
        call(f)
        dts.append(time.perf_counter() - t0)
    dt = float(np.median(dts))
    return {"value": S / dt, "unit": "calls/s", "steps": frames - 2,
            "ms_per_step": 1000 * dt, "ms_per_step_all": [round(1000 * x, 3) for x in dts],
            "note": "host-buffer ABI: packed dets host->device and output rows device->host "
                    "inside every step (pageable numpy buffers); median step"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from yolo_tracking_amd import ByteTrackEngine, _lib
    S, N = args.streams, args.n
    F = args.warmup + args.steps
    Q = max(1, args.queues)
    # with Q > 1 engines, ISO more frames after the timed region run on engine 0 alone: the
    # roofline kernel's rate without the other engines' overlap (reported beside, never `value`)
    ISO = 3 if Q > 1 and not args.no_isolated else 0
    FT = F + ISO
    # synthetic frames for this rank's streams, staged in HBM: [FT][S*N][6] + offsets
    t_gen = time.time()
    per_stream = [gen_stream_frames(N, FT, sd) for sd in stream_seeds(args.seed, rank, S)]
    host = np.stack([np.concatenate([per_stream[s][f] for s in range(S)]) for f in range(FT)])
    counts = np.array([[len(per_stream[s][f]) for s in range(S)] for f in range(FT)])
    off = np.zeros((FT, S + 1), dtype=np.int32)
    np.cumsum(counts, axis=1, out=off[:, 1:])
    del per_stream, counts
    # Q engines (each its own HIP stream) over contiguous slices of the streams: their launches
    # run concurrently, so one engine's latency-bound block chains overlap the other's
    assert S % Q == 0, "--streams must be a multiple of --queues"
    Sq = S // Q
    d_dets, d_off = [], []
    for q in range(Q):
        lo, hi = off[:, q * Sq], off[:, (q + 1) * Sq]
        dq = np.stack([host[f, lo[f]:hi[f]] for f in range(FT)]) if len(set(hi - lo)) == 1 else None
        assert dq is not None, "synthetic frames have N detections per stream"
        d_dets.append(torch.from_numpy(np.ascontiguousarray(dq)).to("cuda"))
        d_off.append(torch.from_numpy(np.ascontiguousarray(off[:, q * Sq:(q + 1) * Sq + 1]
                                                          - off[:, q * Sq:q * Sq + 1])).to("cuda"))
    gen_s = time.time() - t_gen

    engs = [ByteTrackEngine(Sq, track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30,
                            device=local_rank, track_capacity=2 * N, max_dets=N) for _ in range(Q)]
    eng = engs[0]
    cap, _ = eng.capacity()
    d_out = [torch.empty((Sq * cap, 8), dtype=torch.float64, device="cuda") for _ in range(Q)]
    d_cnt = [torch.zeros(Sq, dtype=torch.int32, device="cuda") for _ in range(Q)]
    lib = eng.lib
    handles = [e.handle for e in engs]
    h = handles[0]
    row_bytes = N * 6 * 8 * Sq

    def step(f, engines=None):
        for q in (range(Q) if engines is None else engines):
            _lib.check(lib.yta_bytetrack_update_device(
                handles[q], ctypes.c_void_p(d_dets[q].data_ptr() + f * row_bytes),
                ctypes.c_void_p(d_off[q].data_ptr() + f * (Sq + 1) * 4),
                ctypes.c_void_p(d_out[q].data_ptr()), ctypes.c_void_p(d_cnt[q].data_ptr())))

    def sync_all():
        for hq in handles:
            _lib.check(lib.yta_bytetrack_sync(hq))

    torch.cuda.synchronize()
    for f in range(args.warmup):
        step(f)
    sync_all()
    for hq in handles:
        _lib.check(lib.yta_bytetrack_profile(hq, 1))
    def run_steps():
        for f in range(args.warmup, F):
            step(f)
        sync_all()

    elapsed = timed_region(run_steps, torch.cuda.synchronize, dist)
    # per-launch phase times: engine 0's HIP events (with Q > 1 they overlap the other engines')
    ms = (ctypes.c_double * len(PHASES))()
    nfr = ctypes.c_int()
    _lib.check(lib.yta_bytetrack_profile_collect(h, ms, ctypes.byref(nfr)))
    phase_ms = {PHASES[k]: ms[k] / max(nfr.value, 1) for k in range(len(PHASES))}
    for hq in handles[1:]:
        _lib.check(lib.yta_bytetrack_profile_collect(hq, ms, ctypes.byref(nfr)))
    iso_ms = None
    if ISO:   # after the timed region: engine 0 alone (the other engines idle) for ISO frames
        sync_all()
        for f in range(F, FT):
            step(f, engines=[0])
        _lib.check(lib.yta_bytetrack_profile_collect(h, ms, ctypes.byref(nfr)))
        iso_ms = {PHASES[k]: ms[k] / max(nfr.value, 1) for k in range(len(PHASES))}

    elapsed = max_over_ranks(elapsed, dist, "cuda")
    value = aggregate_rate(world, S, args.steps, elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps

    stats = (ctypes.c_longlong * len(STATS))()
    st = {k: 0 for k in STATS}
    for hq in handles:   # summed over the engines (all S streams)
        _lib.check(lib.yta_bytetrack_stats(hq, stats))
        for k in range(len(STATS)):
            st[STATS[k]] += int(stats[k])
    st_launch = {k: v // Q for k, v in st.items()}   # one engine's launch (Q equal slices)
    if rank == 0:
        # roofline kernel: the longest launch of the frame (the Kalman pass k_apply, HBM-bound)
        dom = max(phase_ms, key=lambda p: phase_ms[p])
        dom_ms = phase_ms[dom]
        b = kernel_bytes(dom, st_launch)
        achieved = b / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        busiest = max(phase_ms, key=lambda p: phase_ms[p])
        per_kernel = {p: {"ms": phase_ms[p], "alg_bytes": kernel_bytes(p, st_launch),
                          "gbs": (kernel_bytes(p, st_launch) / (phase_ms[p] * 1e-3) / 1e9
                                  if phase_ms[p] > 0 else 0.0)} for p in PHASES}
        cpu = None if args.no_cpu_baseline else cpu_baseline(N, args.cpu_frames, args.seed)
        pcie = None if args.no_pcie else pcie_inclusive(host, off, S, N, local_rank)
        traffic, step_traffic, traffic_tag = pmc_traffic(S, N, Q)
        line = {
            "metric": "tracker.update() calls/sec @ 1024 tracks×1024 dets; 1/2/4/8 MI355X",
            "value": value, "unit": "calls/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"bytetrack {N}x{N}, {S} streams/GPU, inputs resident in HBM",
                       "tracker": "bytetrack", "tracks": N, "dets": N, "streams_per_gpu": S,
                       "queues_per_gpu": Q, "parallelism": f"stream-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": (f"profiles/{traffic_tag}_summary.json (rocprofv3 "
                                            "FETCH_SIZE x2 + WRITE_SIZE)" if traffic else None),
                         "algorithmic_bytes_per_launch": b, "avg_launch_ms": dom_ms,
                         "launch_streams": S // Q,
                         # every kernel of every engine: measured HBM bytes per step / step time
                         "chip_gbs": (step_traffic / (ms_per_step * 1e-3) / 1e9
                                      if step_traffic else None),
                         "isolated": (None if iso_ms is None else {
                             "avg_launch_ms": iso_ms[dom],
                             "achieved": b / (iso_ms[dom] * 1e-3) / 1e9,
                             "frac": b / (iso_ms[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "frames": ISO,
                             "note": "engine 0 alone for the frames after the timed region, "
                                     "same algorithmic bytes per launch"}),
                         "note": (None if Q == 1 else
                                  f"{Q} engines of {S // Q} streams on {Q} HIP streams: each "
                                  "launch overlaps the other engines' kernels, so its duration "
                                  "(and this per-launch rate) includes their share of the chip")},
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "per_kernel": per_kernel,
            "frame_counts": st,
            "busiest_kernel": busiest,
            "single_stream_equiv_ms": ms_per_step,
            "algorithmic_bytes_per_update": algorithmic_bytes(N, N),
            "stage_seconds": round(gen_s, 1),
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
