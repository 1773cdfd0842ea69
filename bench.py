#!/usr/bin/env python3
"""Throughput of the MI355X ByteTrack update() (BASELINE.json headline metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--streams S] [--n 1024]

A step = one `tracker.update()` frame for every one of the S independent streams on each GPU
(each stream: 1024 tracks x 1024 detections per frame, SURVEY.md §8(d) synthetic generator).
All frames are staged in HBM before the timed region; the engine's device-buffer entry point
runs the whole update on the GPU (outputs stay in HBM).  Before the W warmup frames, `--preroll`
frames (default 35 > max_time_lost = 30, byte_tracker.py:128-129) run untimed, so the timed
frames see the steady state: Lost tracks expire as fast as they are created.

N > 1: one process per GPU, streams sharded per rank with disjoint seeds, no data-path
collective, barrier + max over ranks around the timed region (scaling "weak": per-GPU work is
fixed).  Launched either by torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE in the
environment) or directly as `bench.py --gpus N`: the parent then starts N rank processes itself
(before it touches torch or the GPU) and waits for them, the way examples/val.py:147-226 starts one
process per sequence and device.  `--dry-cpu` runs the same harness on CPU ranks over gloo with a
NumPy stand-in step (tests/test_bench_harness.py).

Rank 0 prints one JSON line with `roofline` (the longest launch of the isolated leg - engine 0
alone after the timed region - by HIP events on its stream, with its measured HBM bytes from the
committed rocprofv3 PMC summary, per kernel),
`pcie_inclusive` (host buffers in and out every call) and `cpu_baseline` (the oracle's CPU
restatement on this host: 1 core and all cores, bounded sample).
"""
import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PHASES = ["s1_prep", "s1_edges", "s1_lap", "stage23", "apply", "finish"]
STATS = ["dets", "high", "second", "pool", "act", "unc", "left", "rest", "births", "t2", "l2",
         "tracked", "lost", "out", "edges1", "edges23", "fallback1", "fallback23", "lazy", "res1",
         "fallback_f"]
# yta_bytetrack_pipe_stats slots (bench reports them per frame, "frames" as the total)
PIPE_STATS = ["frames", "in_direct_bytes", "in_staged_bytes", "out_direct_bytes", "out_staged_bytes",
              "host_stage_in_ms", "host_submit_ms", "host_wait_ms", "host_copy_out_ms",
              "gpu_in_ms", "gpu_kernels_ms", "gpu_out_ms", "gpu_span_ms", "host_h2d_call_ms",
              "host_launch_ms", "host_d2h_call_ms", "host_small_h2d_ms", "host_small_d2h_ms",
              "host_pinned_check_ms", "capacity_waits", "capacity_drains"]
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Canonical algorithmic bytes per update: ByteTrack 1024 x 1024
BYTES_PER_UPDATE_1024 = 19_259_392


def algorithmic_bytes(n, m):
    """B = 4*S*N + 56*M + 16*N*M + 64*N with S = 576 (ByteTrack)."""
    return 4 * 576 * n + 56 * m + 16 * n * m + 64 * n


def kernel_bytes(phase, st, slots=0):
    """Algorithmic HBM bytes one launch of `phase` must move: every array element the kernel has
    to read or write once, from the last frame's counts summed over the launch's streams
    (csrc/bytetrack.hip).  Kalman state = 24 f64 (192 B), track meta = 48 B,
    box = 32 B, detection row = 48 B (6 f64), list entry / index = 4 B, candidate edge = 12 B (int
    column + f64 cost).  slots: S * track capacity of the launch (k_finish rewrites the free list).
    Line granularity (a 32-B box read moves a 128-B line) and whole-line record writes are not
    algorithmic: they show as counter bytes above these (`pmc_over_alg` > 1)."""
    pool, unc, high, dets = st["pool"], st["unc"], st["high"], st["dets"]
    act, lazy, second, left, rest = st["act"], st["lazy"], st["second"], st["left"], st["rest"]
    births, t2, l2, out = st["births"], st["t2"], st["l2"], st["out"]
    tracked, lost = st["tracked"], st["lost"]
    lost_pool = pool - act              # the pool's tail: the previous frame's lost list
    refound = max(lost_pool - lazy, 0)  # lost tracks matched in stage 1
    updated = max(t2 - births, 0)       # tracks that took a detection (tracked' minus births)
    if phase == "s1_prep":
        # detection rows read; high list (index, box, score) and low list (index, box) written
        # (the pool itself is built by the previous frame's k_finish)
        return dets * 48 + high * (4 + 32 + 8) + second * (4 + 32)
    if phase == "s1_edges":
        # high boxes + scores read once (grid built in LDS), y1 written per high detection; every
        # pool box read, edge count and single-edge result x1 written per row; edge slots written
        return high * (32 + 8 + 4) + pool * (32 + 4 + 4) + st["edges1"] * 12
    if phase == "s1_lap":
        # every pool row's edge count; the residual rows' edges (after the single-edge
        # components) read; their matches written (x1 / y1, at most one per residual edge)
        return pool * 4 + st["res1"] * (12 + 8)
    if phase == "stage23":
        # left_of_pool reset, stage-1 results of the pool head (leftovers) and tail (re-found:
        # slot + result read, pair written), y1 of the high detections (rest), rest entries with
        # scores; stage 2: leftover boxes x low boxes, x2 / y2; stage 3: unconfirmed boxes x rest
        # boxes + scores, x3 / y3
        return (pool * 4 + act * 4 + lost_pool * 8 + refound * 8 + high * 4
                + left * (4 + 32 + 4) + second * (32 + 4)
                + rest * (4 + 8 + 8) + unc * (32 + 4) + rest * (4 + 32 + 8 + 4))
    if phase == "apply":
        # every pool / unconfirmed item: slot + stage results; every track but the lazily
        # predicted lost ones: flags, Kalman state + meta read, Kalman state written; tracks that
        # took a detection: meta written, the detection's row + its list index read
        touched = pool - lazy + unc
        return (pool * 12 + unc * 8 + touched * (4 + 192 + 48 + 192) + updated * (48 + 48 + 4))
    if phase == "finish":
        # births: rest entries (result, score, index, high index); per birth: free slot, detection
        # row, Kalman state + meta + flags written.  tracked' = previous tracked list (slot, flags)
        # ++ births ++ re-found; lost' = previous lost list (slot, flags, lost frame) ++ leftovers
        # (result, position, slot, flags); duplicate removal: lost' pool boxes, tracked' boxes;
        # final lists (tracked' flags, tracked / lost / unconfirmed written); output rows: mean +
        # meta read, row written, and the next frame's pool: head boxes, unconfirmed boxes, the
        # lost tail (mean, flags, lost frame) predicted; the free list rewritten
        free = max(slots - tracked - lost, 0)
        return (rest * (4 + 8 + 4 + 4) + births * (4 + 4 + 48 + 192 + 48 + 4)
                + (act + st["unc"]) * 8 + t2 * 4 + births * 4 + refound * 8
                + lost_pool * 12 + left * 16 + l2 * 8
                + l2 * (4 + 32) + t2 * (4 + 32)
                + t2 * (4 + 4) + tracked * 4 + l2 * 4 + lost * 4
                + out * (4 + 64 + 48) + out * (64 + 4 + 32)
                + (tracked - out) * (4 + 32 + 4 + 32)
                + lost * (4 + 64 + 4 + 4) + lost * (4 + 32)
                + free * 4)
    return 0


PHASE_KERNEL = {"s1_prep": "k_s1_prep", "s1_edges": "k_s1_edges", "s1_lap": "k_s1_lap",
                "stage23": "k_stage23", "apply": "k_apply", "finish": "k_finish"}


def pmc_traffic(streams, n, queues):
    """Measured HBM bytes per launch of every kernel of the frame, and per step of the whole frame
    (every kernel of every engine), from the committed rocprofv3 PMC summary
    (profiles/roofline_traffic.json, written by profiles/summarize.py: FETCH_SIZE x 2 +
    WRITE_SIZE in separate passes, keyed by kernel), when it was measured on this same workload;
    else ({}, None, None)."""
    f = os.path.join(REPO, "profiles", "roofline_traffic.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return {}, None, None
    if (d.get("streams") == streams and d.get("n") == n and d.get("queues", 1) == queues
            and isinstance(d.get("kernels"), dict)):
        return d["kernels"], d.get("hbm_bytes_per_step"), d.get("tag")
    return {}, None, None


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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--preroll", type=int, default=35,
                   help="untimed frames before the warmup (steady state: > max_time_lost = 30)")
    p.add_argument("--streams", type=int, default=None,
                   help="streams per GPU (default: bytetrack 2048; the other trackers their "
                        "config's per-GPU share, CONFIG_SHARE)")
    p.add_argument("--n", type=int, default=None,
                   help="tracks = detections per frame (default: bytetrack 1024; the other "
                        "trackers their config's size)")
    p.add_argument("--tracker", default="bytetrack",
                   choices=["bytetrack", "ocsort", "botsort", "deepocsort", "hybridsort"],
                   help="bytetrack: the headline (BASELINE.json metric); the others run their "
                        "BASELINE config (C2-C5) as the measured workload, streams sharded s mod "
                        "G over the ranks (tools/bench_tracker.py engines)")
    p.add_argument("--dim", type=int, default=512, help="embedding width (ReID trackers)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe) leg")
    p.add_argument("--pcie-engines", type=int, default=1,
                   help="engines (host threads) of the host-buffer leg")
    p.add_argument("--no-pcie-pinned", action="store_true",
                   help="skip the host-buffer leg's page-locked variant")
    p.add_argument("--no-dropin", action="store_true", help="skip the one-stream drop-in leg")
    p.add_argument("--no-configs", action="store_true", help="skip the configs C2-C5 legs")
    p.add_argument("--no-isolated", action="store_true",
                   help="skip the engine-0-alone frames after the timed region (profiling runs)")
    p.add_argument("--cpu-frames", type=int, default=40)
    p.add_argument("--seed", type=int, default=1000)
    p.add_argument("--queues", type=int, default=2,
                   help="engines per GPU, each on its own HIP stream, streams split between them")
    p.add_argument("--shared-gpu", action="store_true",
                   help="rehearsal on a box with fewer GPUs than ranks: rank r uses device "
                        "r mod device_count and the ranks synchronise over gloo (not a scaling "
                        "measurement: the ranks share the card)")
    p.add_argument("--dry-cpu", action="store_true",
                   help="harness rehearsal: CPU ranks over gloo, NumPy stand-in step, no GPU")
    a = p.parse_args(argv)
    if a.tracker == "bytetrack":
        a.streams = 2048 if a.streams is None else a.streams
        a.n = 1024 if a.n is None else a.n
    else:
        a.streams = CONFIG_SHARE[a.tracker][1] if a.streams is None else a.streams
        a.n = CONFIG_SHARE[a.tracker][0] if a.n is None else a.n
    return a


# BASELINE.json configs of the other trackers: (tracks = dets, streams per GPU).  C4 = 8 DeepOCSORT
# streams over 8 GPUs (1 per GPU), C5 = 64 HybridSORT streams over 8 GPUs (8 per GPU); C2 / C3
# are single-GPU configs (1 stream).  With --gpus G every GPU runs this share (weak scaling), so
# G = 8 is the config as BASELINE states it.
CONFIG_SHARE = {"ocsort": (256, 1), "botsort": (1024, 1), "deepocsort": (2048, 1),
                "hybridsort": (4096, 8)}


def config_seeds(seed, rank, world, streams):
    """Stream s of the job -> rank s mod G (examples/val.py:147-226 hands sequences to devices in
    turn); rank r's k-th stream is global stream r + k G, seeded seed + r + k G."""
    return [seed + rank + world * k for k in range(streams)]


# ---------------------------------------------------------------- rank launcher (--gpus N)
def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, n):
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), wait
    for all of them, and return the first non-zero exit status.  Runs before anything touches
    torch or the GPU; if one rank fails the others are stopped (they would wait at a barrier)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def peak_rss_mb():
    """This process's peak resident set (MB), before the rank-0-only PCIe / CPU legs."""
    import resource
    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0, 1)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or None


def cpu_share():
    """Host cores this job may use: the affinity mask, capped by OMP_NUM_THREADS when the
    environment sets it (16 per GPU on the GPU box)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def gen_stream_frames(n, frames, seed):
    from yolo_tracking_amd.synth import make_frames
    return [d for d, _ in make_frames(n, frames, seed)]


def stage_frames(n, frames, seeds, Q, device):
    """Synthetic frames of this rank's streams straight into HBM, one frame at a time: every
    stream's generator advances one frame into a page-locked [S*N][6] buffer, which is copied into
    each engine's [frames][S/Q*N][6] device tensor.  Host memory stays at one frame of every
    stream (no per-stream frame lists, no stacked copy), whatever the step count or rank count.
    Returns (per-engine device tensors, per-engine device offset tensors [frames][S/Q + 1])."""
    import torch

    from yolo_tracking_amd.synth import SyntheticStream
    S = len(seeds)
    Sq = S // Q
    gens = [SyntheticStream(n, sd) for sd in seeds]
    buf = torch.empty((S * n, 6), dtype=torch.float64, pin_memory=True)
    host = buf.numpy()
    d_dets = [torch.empty((frames, Sq * n, 6), dtype=torch.float64, device=device)
              for _ in range(Q)]
    for f in range(frames):
        for s, g in enumerate(gens):
            d, _ = g.next_frame()
            assert len(d) == n, "synthetic frames have N detections per stream"
            host[s * n:(s + 1) * n] = d
        for q in range(Q):
            d_dets[q][f].copy_(buf[q * Sq * n:(q + 1) * Sq * n])
    torch.cuda.synchronize()
    off = torch.arange(Sq + 1, dtype=torch.int32) * n
    d_off = [off.repeat(frames, 1).contiguous().to(device) for _ in range(Q)]
    return d_dets, d_off


_CPU_LEG = (
    "import sys,time,json; sys.path.insert(0,%r)\n"
    "from oracle.bytetrack import ByteTrackOracle\n"
    "from yolo_tracking_amd.synth import make_frames\n"
    "fr=[d for d,_ in make_frames(%d,%d,%d)]\n"
    "t=ByteTrackOracle(0.5,0.8,30,30); t.update(fr[0])\n"
    "t0=time.perf_counter()\n"
    "for d in fr[1:]: t.update(d)\n"
    "dt=time.perf_counter()-t0\n"
    "print(json.dumps({'frames':len(fr)-1,'seconds':dt}))\n")


def cpu_baseline(n, frames, seed):
    """Time the oracle (CPU restatement: NumPy ByteTrack + C lapjv, the cpu_baseline leg is the
    only place bench.py runs it) on this host: one stream on 1 thread, then one stream per core
    of this job's CPU share, all at once (1 core + all cores, CPU model)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    P = cpu_share()

    def start(sd):
        return subprocess.Popen([sys.executable, "-c", _CPU_LEG % (REPO, n, frames, sd)], env=env,
                                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)

    def result(proc):
        out, _ = proc.communicate(timeout=900)
        return json.loads(out.strip().splitlines()[-1])

    base = {"unit": "calls/s", "kind": "port", "cpu_model": cpu_model()}
    try:
        one = result(start(seed))
    except Exception as exc:  # report, never fail the bench on the baseline leg
        return dict(base, value=None, cores=1, sample=f"failed: {exc}")
    line = dict(base, value=one["frames"] / one["seconds"], cores=1,
                sample=f"oracle ByteTrack (NumPy + C lapjv), 1 stream {n}x{n}, frames 2..{frames} "
                       f"of seed {seed}, {one['seconds']:.1f} s, 1 thread")
    try:
        res = [result(p) for p in [start(seed + k) for k in range(P)]]
        line["all_cores"] = {
            "value": sum(r["frames"] for r in res) / max(r["seconds"] for r in res),
            "cores": P, "processes": P,
            "sample": f"{P} processes at once, one stream each (seeds {seed}..{seed + P - 1}), "
                      f"frames 2..{frames}, 1 thread each; total frames / slowest process"}
    except Exception as exc:
        line["all_cores"] = {"value": None, "cores": P, "sample": f"failed: {exc}"}
    return line


def pinned_empty(shape, dtype):
    """A page-locked host array (torch's pinned allocator), as a detector writing its boxes into
    pinned memory would hand it over.  tools/pipe_probe.py swaps in other allocators."""
    import torch
    return torch.empty(shape, dtype=torch.float32 if dtype == np.float32 else torch.float64,
                       pin_memory=True).numpy()


def pcie_inclusive(frame_of, S, N, device, first, frames=8, engines=1, pinned=False):
    """The same workload through the host-buffer ABI (yta_bytetrack_update: packed host dets in,
    output rows back to the host every call, synchronous) on fresh engines, frames 0..first-1
    untimed (steady state), then `frames` timed steps: rank 0's report of the PCIe-inclusive
    rate.  frame_of(f) -> the (S*N, 6) host array of frame f (read back from the staged device
    frames, untimed).  With engines > 1 the streams are split over that many engines whose calls
    run on as many host threads at once (ctypes releases the GIL), so one engine's copies overlap
    another's kernels, as a multi-camera host would run them; a step ends when every engine's call
    has returned.  pinned: the caller's buffers are page-locked (as a detector writing its boxes
    into pinned memory would leave them): each frame's dets are placed in them before its timed
    call, and the library DMAs straight from / into them (no staging copy).  Never `value`
    (DESIGN.md §5)."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    from yolo_tracking_amd import ByteTrackEngine, _lib
    E = max(1, min(engines, S))
    bounds = [S * q // E for q in range(E + 1)]
    engs, jobs = [], []

    def buf(shape):
        if not pinned:
            return np.empty(shape)
        return pinned_empty(shape, np.float64)
    for q in range(E):
        a, b = bounds[q], bounds[q + 1]
        # capacity 3N: the host path reserves ahead of need (tracked + lost + this frame's dets,
        # ~2.2N in the steady state) and would otherwise regrow the engine on the first frames
        eng = ByteTrackEngine(b - a, track_thresh=0.5, match_thresh=0.8, track_buffer=30,
                              frame_rate=30, device=device, track_capacity=3 * N, max_dets=N)
        engs.append(eng)
        jobs.append({"h": eng.handle, "lib": eng.lib, "a": a, "b": b,
                     "offs": np.ascontiguousarray(np.arange(b - a + 1, dtype=np.int32) * N),
                     "out": buf(((b - a) * N, 8)), "out_off": np.zeros(b - a + 1, np.int32),
                     "nid": np.zeros(b - a, np.int64), "in": buf(((b - a) * N, 6))})
    last = first + frames

    def place(f):   # this frame's dets into the callers' buffers (untimed)
        fr = frame_of(f)
        for j in jobs:
            j["in"][:] = fr[j["a"] * N:j["b"] * N]

    def call(j):
        _lib.check(j["lib"].yta_bytetrack_update(j["h"], j["in"].ctypes.data,
                                                 j["offs"].ctypes.data, j["nid"].ctypes.data,
                                                 j["out"].ctypes.data, len(j["out"]),
                                                 j["out_off"].ctypes.data))
    pool = ThreadPoolExecutor(max_workers=E)

    def step():
        if E == 1:
            call(jobs[0])
        else:
            for r in [pool.submit(call, j) for j in jobs]:
                r.result()
    for f in range(first):
        place(f)
        step()
    dts = []
    for f in range(first, last):
        place(f)
        t0 = time.perf_counter()
        step()
        dts.append(time.perf_counter() - t0)
    pool.shutdown()
    dt = float(np.median(dts))
    return {"value": S / dt, "unit": "calls/s", "steps": len(dts), "untimed_frames": first,
            "engines": E, "ms_per_step": 1000 * dt,
            "ms_per_step_all": [round(1000 * x, 3) for x in dts],
            "bytes_h2d_per_step": S * N * 48,
            "note": "host-buffer ABI: packed dets host->device and output rows device->host "
                    f"inside every step ({'page-locked' if pinned else 'pageable numpy'} buffers, "
                    f"{E} engine(s) on as many host threads); median step"}


def pcie_pipelined(frame_of, S, N, device, first, frames=8, pinned=False, f32=False, cap_mult=3,
                   check=None, offsets_of=None):
    """The host-buffer path pipelined (yta_bytetrack_submit / _collect, one engine): frame f's
    detections go host -> device while frame f-1's kernels run and frame f-2's rows come back (up
    to three frames in flight), so both PCIe directions and the kernels overlap.  Every timed frame's packed dets sit in their
    own caller buffer before the timed region (page-locked: written there by the detector, DMA'd
    directly; pageable: staged by the library during submit); output rows land in three
    rotating caller buffers (page-locked: DMA'd directly).  value = frames / wall time of the
    timed submit/collect loop.  Never `value` of the bench line.

    Parity hooks (tests/test_gpu_pipelined_bench_shape.py runs this very function):
    offsets_of(f) -> the S + 1 detection offsets of frame f (default: N rows per stream);
    check(f, rows, out_off) is called after each collect with frame f's packed output rows (a view
    of the caller buffer) and offsets, and check(None, next_ids, pipe_stats) once at the end."""
    import torch

    from yolo_tracking_amd import ByteTrackEngine, _lib
    eng = ByteTrackEngine(S, track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30,
                          device=device, track_capacity=cap_mult * N, max_dets=N)
    lib, h = eng.lib, eng.handle

    def buf(shape, dt=np.float64):
        if not pinned:
            return np.empty(shape, dtype=dt)
        return pinned_empty(shape, dt)
    uniform = np.ascontiguousarray(np.arange(S + 1, dtype=np.int32) * N)
    offs_all = [uniform if offsets_of is None else
                np.ascontiguousarray(offsets_of(f), dtype=np.int32) for f in range(first + frames)]
    rows_max = max(int(o[-1]) for o in offs_all)
    in_dt = np.float32 if f32 else np.float64
    submit_fn = lib.yta_bytetrack_submit_f32 if f32 else lib.yta_bytetrack_submit
    # frames in flight (csrc/bytetrack.hip PIPE_DEPTH; YTA_PIPE_DEPTH names a -DYTA_PIPE_DEPTH
    # variant library's depth for A/B runs)
    DEPTH = int(os.environ.get("YTA_PIPE_DEPTH", "3"))
    outs = [buf((rows_max, 8)) for _ in range(DEPTH)]
    out_off = np.zeros(S + 1, np.int32)
    stage = buf((rows_max, 6), in_dt)
    inflight = []

    def submit(src, f):
        o = offs_all[f]
        _lib.check(submit_fn(h, src.ctypes.data, o.ctypes.data, None,
                             outs[f % DEPTH].ctypes.data, rows_max))
        inflight.append(f)

    def collect():
        _lib.check(lib.yta_bytetrack_collect(h, None, out_off.ctypes.data))
        f = inflight.pop(0)
        if check is not None:
            check(f, outs[f % DEPTH][:out_off[-1]], out_off.copy())
    for f in range(first):   # untimed: steady state
        n = int(offs_all[f][-1])
        stage[:n] = frame_of(f)
        submit(stage, f)
        collect()
    timed = []
    for f in range(first, first + frames):
        n = int(offs_all[f][-1])
        b = buf((n, 6), in_dt)
        b[:] = frame_of(f)
        timed.append(b)
    _lib.check(lib.yta_bytetrack_pipe_stats(h, None, 0, 1))   # accounting from here
    t0 = time.perf_counter()
    for k, src in enumerate(timed):
        submit(src, first + k)
        if k >= DEPTH - 1:
            collect()
    for _ in range(min(DEPTH - 1, len(timed))):
        collect()
    dt = (time.perf_counter() - t0) / frames
    ps = (ctypes.c_double * len(PIPE_STATS))()
    _lib.check(lib.yta_bytetrack_pipe_stats(h, ps, len(PIPE_STATS), 1))
    nfr = max(ps[0], 1.0)
    acct = {k: (ps[i] / nfr if i else ps[i]) for i, k in enumerate(PIPE_STATS)}
    if check is not None:
        nid = np.zeros(S, np.int64)
        _lib.check(lib.yta_bytetrack_next_ids(h, nid.ctypes.data))
        check(None, nid, {k: ps[i] for i, k in enumerate(PIPE_STATS)})
    eng.close()
    return {"value": S / dt, "unit": "calls/s", "steps": frames, "ms_per_step": 1000 * dt,
            "per_frame": {k: round(v, 4) for k, v in acct.items()},
            "note": "pipelined host-buffer ABI (submit/collect, up to three frames in flight), "
                    f"{'page-locked' if pinned else 'pageable numpy'} caller buffers"
                    f"{', float32 detection rows' if f32 else ''}; "
                    "wall time of the timed loop / frames"}


def dropin_leg(n, frames, seed, device):
    """North star's per-stream claim: one camera stream through the reference's plugin surface,
    exactly as examples/track.py:43-57 drives it - create_tracker('bytetrack', ...) then
    tracker.update(dets, img) with NumPy in and out every call (float32 boxes, as ultralytics hands
    them over; host -> device, kernels, device -> host inside every call).  Median over frames
    2..frames.  Beside it in the line: the 1-core oracle on the same workload
    (cpu_baseline)."""
    from yolo_tracking_amd import create_tracker, get_tracker_config
    from yolo_tracking_amd.synth import make_frames
    fr = [d.astype(np.float32) for d, _ in make_frames(n, frames, seed)]
    img = np.zeros((8, 8, 3), np.uint8)     # ignored by ByteTrack (byte_tracker.py:132)
    t = create_tracker("bytetrack", get_tracker_config("bytetrack"), None, device, False, False)
    dts, rows = [], 0
    for d in fr:
        t0 = time.perf_counter()
        out = t.update(d, img)
        dts.append(time.perf_counter() - t0)
        rows = len(out)
    med = float(np.median(dts[1:]))
    return {"value": 1.0 / med, "unit": "calls/s", "median_ms": 1e3 * med,
            "p90_ms": 1e3 * float(np.percentile(dts[1:], 90)), "frames": f"2..{frames}",
            "rows_last_frame": rows,
            "workload": f"bytetrack {n}x{n}, one stream, create_tracker + update(dets, img), "
                        "float32 NumPy dets in, (K, 8) float64 NumPy rows out per call"}


# configs 2-5 (BASELINE.json configs[1..4]) at their stated sizes, single GPU: tools/bench_tracker.py
CONFIGS = [
    ("C2", ["--tracker", "ocsort", "--n", "256", "--streams", "1", "--steps", "50"]),
    ("C3", ["--tracker", "botsort", "--n", "1024", "--dim", "512", "--streams", "1",
            "--steps", "30"]),
    ("C4", ["--tracker", "deepocsort", "--n", "2048", "--dim", "512", "--streams", "1",
            "--steps", "20"]),
    ("C5", ["--tracker", "hybridsort", "--n", "4096", "--dim", "512", "--streams", "8",
            "--steps", "8", "--warmup", "3"]),
]


def configs_leg(names=None):
    """Configs C2-C5 on this GPU (tools/bench_tracker.py: inputs staged in HBM, the engines'
    device-buffer entry points, timed frames between device syncs), each with its 1-core oracle
    (started together beside the GPU legs, collected after).  C5 runs its per-GPU share of the
    64-stream config: 8 streams in two engines.  names: a subset (N > 1 ranks: C2 / C3, the
    single-GPU configs; C4 / C5 then run on every rank, MULTI_CONFIGS)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_tracker as bt
    todo = [(name, bt.parse(argv)) for name, argv in CONFIGS if names is None or name in names]
    cpus = {name: bt.start_cpu_leg(a) for name, a in todo}
    res = {}
    for name, a in todo:
        t0 = time.time()
        try:
            line = bt.run(a, cpu=cpus[name])
        except Exception as exc:   # report, never fail the bench on a config leg
            res[name] = {"value": None, "error": repr(exc)[:300]}
            continue
        cpu = line.get("cpu_baseline") or {}
        res[name] = {"metric": line["metric"], "value": line["value"], "unit": "calls/s",
                     "ms_per_step": line["ms_per_step"], "steps": line["steps"],
                     "workload": line["config"]["workload"], "cpu_1core": cpu.get("value"),
                     "cpu_sample": cpu.get("sample"),
                     "vs_cpu_1core": (line["value"] / cpu["value"] if cpu.get("value") else None),
                     "wall_s": round(time.time() - t0, 1)}
    return res


def run_dry(args, world, rank):
    """--dry-cpu: the multi-rank harness end to end on CPU ranks (gloo): stream sharding, frame
    staging, barrier-bracketed timed region, max over ranks, rank-0 JSON line.  The step is a
    NumPy stand-in over the staged frames (no GPU, no tracker).  With --tracker other than
    bytetrack: that config's streams (embeddings for the ReID trackers), sharded s mod G."""
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    S, N = args.streams, args.n
    cfg = args.tracker != "bytetrack"
    seeds = config_seeds(args.seed, rank, world, S) if cfg else stream_seeds(args.seed, rank, S)
    F = (0 if cfg else args.preroll) + args.warmup + args.steps
    if cfg and args.tracker != "ocsort":
        from yolo_tracking_amd.synth import make_frames
        frames = [make_frames(N, F, sd, emb_dim=args.dim) for sd in seeds]
    else:
        frames = [[(d, None) for d in gen_stream_frames(N, F, sd)] for sd in seeds]
    acc = np.zeros(S)

    def step(f):
        for s in range(S):
            d, e = frames[s][f]
            acc[s] += d[:, 4].sum() + (float(e[:, 0].sum()) if e is not None else 0.0)

    for f in range(F - args.steps):
        step(f)

    def run_steps():
        for f in range(F - args.steps, F):
            step(f)

    elapsed = timed_region(run_steps, lambda: None, dist)
    elapsed = max_over_ranks(elapsed, dist, "cpu")
    every = [seeds]
    if dist:
        every = [None] * world
        dist.all_gather_object(every, seeds)
    if rank == 0:
        print(json.dumps({"metric": "dry-run harness", "value": aggregate_rate(world, S, args.steps,
                                                                              elapsed),
                          "unit": "calls/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "tracker": args.tracker,
                          "tracks": N, "streams_per_gpu": S, "stream_seeds_by_rank": every,
                          "checksum": float(acc.sum())}))
    if dist:
        dist.destroy_process_group()


def config_shard_leg(tracker, n, dim, streams, steps, warmup, seed, world, rank, dist, device,
                     cpu=False):
    """One BASELINE config on every rank at once (tools/bench_tracker.py's engines, inputs staged in
    HBM): rank r runs `streams` streams, global streams r, r + G, ... (s mod G); the timed region
    is bracketed by the ranks' barrier, the job's time is the slowest rank's, value = all ranks'
    update calls / that time.  cpu: the 1-core oracle beside it (rank 0, N = 1 only)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_tracker as bt
    argv = ["--tracker", tracker, "--n", str(n), "--streams", str(streams), "--steps", str(steps),
            "--warmup", str(warmup), "--seed", str(seed)]
    if tracker != "ocsort":
        argv += ["--dim", str(dim)]
    a = bt.parse(argv)
    seeds = config_seeds(seed, rank, world, streams)
    cpu_proc = bt.start_cpu_leg(a) if cpu and rank == 0 else (None, 0)
    line = bt.run(a, cpu=cpu_proc, seeds=seeds, barrier=(dist.barrier if dist else None))
    el = max_over_ranks(line["elapsed_s"], dist, device)
    every = [seeds]
    if dist:
        every = [None] * world
        dist.all_gather_object(every, seeds)
    return {"metric": f"{tracker} tracker.update() calls/sec @ {n} tracks x {n} dets",
            "value": aggregate_rate(world, streams, steps, el), "unit": "calls/s",
            "n_gpus": world, "streams_per_gpu": streams, "streams_total": world * streams,
            "steps": steps, "warmup": warmup, "ms_per_step": 1000.0 * el / steps,
            "scaling": "weak", "sharding": "stream s -> rank s mod G",
            "stream_seeds_by_rank": every, "workload": line["config"]["workload"],
            "queues_per_gpu": line["config"].get("queues"),
            "cpu_baseline": line.get("cpu_baseline") if cpu else None,
            "frame_counts_rank0": line.get("frame_counts")}


def run_config(args, world, rank, local_rank):
    """--tracker other than bytetrack: that BASELINE config is the measured workload (C4: one
    DeepOCSORT stream of 2048 x 2048 + CMC per GPU, C5: eight HybridSORT streams of 4096 x 4096 per
    GPU; 8 GPUs = the config as stated), one JSON line on rank 0."""
    import torch
    if args.shared_gpu:   # rehearsal: ranks share the box's card(s), gloo between them
        local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.shared_gpu:   # RCCL refuses two ranks on one device
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    line = config_shard_leg(args.tracker, args.n, args.dim, args.streams, args.steps, args.warmup,
                            args.seed, world, rank, dist, "cpu" if args.shared_gpu else "cuda",
                            cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0:
        line.update(higher_is_better=True, vs_baseline=None, dtype="f64", data="synthetic",
                    config={"workload": line.pop("workload"), "tracker": args.tracker,
                            "tracks": args.n, "dets": args.n, "streams_per_gpu": args.streams,
                            "parallelism": f"stream-sharded x{world}"})
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


# C4 / C5 in the default (headline) run with N > 1 ranks: every rank runs its share at once
MULTI_CONFIGS = [("C4", "deepocsort", 2048, 1, 20, 5), ("C5", "hybridsort", 4096, 8, 8, 3)]


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: using {world} ranks",
              file=sys.stderr)
    if args.dry_cpu:
        return run_dry(args, world, rank)
    if args.tracker != "bytetrack":
        return run_config(args, world, rank, local_rank)
    import torch
    if args.shared_gpu:
        local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.shared_gpu:   # RCCL refuses two ranks on one device
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from yolo_tracking_amd import ByteTrackEngine, _lib
    S, N = args.streams, args.n
    PRE = args.preroll + args.warmup          # untimed frames before the timed region
    F = PRE + args.steps
    Q = max(1, args.queues)
    # with Q > 1 engines, ISO more frames after the timed region run on engine 0 alone: the
    # roofline kernel's launch with the chip to itself (never part of `value`)
    ISO = 3 if Q > 1 and not args.no_isolated else 0
    FT = F + ISO
    # synthetic frames for this rank's streams, staged in HBM one frame at a time:
    # Q x [FT][S/Q*N][6] + offsets
    assert S % Q == 0, "--streams must be a multiple of --queues"
    Sq = S // Q
    t_gen = time.time()
    d_dets, d_off = stage_frames(N, FT, stream_seeds(args.seed, rank, S), Q, "cuda")
    gen_s = time.time() - t_gen

    def frame_of(f):   # the host copy of frame f (pcie leg only; untimed)
        return torch.cat([d[f] for d in d_dets]).cpu().numpy()

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
    for f in range(PRE):
        step(f)
    sync_all()
    for hq in handles:
        _lib.check(lib.yta_bytetrack_profile(hq, 1))

    def run_steps():
        for f in range(PRE, F):
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
    # counters of the last timed frame (summed over the engines: all S streams)
    stats = (ctypes.c_longlong * len(STATS))()
    st = {k: 0 for k in STATS}
    for hq in handles:
        _lib.check(lib.yta_bytetrack_stats(hq, stats))
        for k in range(len(STATS)):
            st[STATS[k]] += int(stats[k])
    iso_ms, st_iso = None, None
    if ISO:   # after the timed region: engine 0 alone (the other engines idle) for ISO frames
        sync_all()
        for f in range(F, FT):
            step(f, engines=[0])
        _lib.check(lib.yta_bytetrack_profile_collect(h, ms, ctypes.byref(nfr)))
        iso_ms = {PHASES[k]: ms[k] / max(nfr.value, 1) for k in range(len(PHASES))}
        _lib.check(lib.yta_bytetrack_stats(h, stats))   # engine 0's last isolated frame
        st_iso = {STATS[k]: int(stats[k]) for k in range(len(STATS))}

    elapsed = max_over_ranks(elapsed, dist, "cpu" if args.shared_gpu else "cuda")
    value = aggregate_rate(world, S, args.steps, elapsed)
    # host memory of every rank after staging and the timed region (the frames live in HBM; the
    # host holds one frame of every stream while staging): peak RSS per rank, in MB
    rss = [peak_rss_mb()]
    if dist:
        rss = [None] * world
        dist.all_gather_object(rss, peak_rss_mb())
    ms_per_step = 1000.0 * elapsed / args.steps
    # N > 1: C4 / C5 with every rank running its share at once (weak scaling: 8 ranks = the
    # configs as BASELINE.json states them); one failing rank would leave the others at a barrier,
    # so a failure is reported, not raised, and the legs run only while every rank is healthy
    multi_cfg = None
    if world > 1 and not args.no_configs:
        multi_cfg = {}
        for name, tr, n, sp, stp, wu in MULTI_CONFIGS:
            try:
                multi_cfg[name] = config_shard_leg(tr, n, 512, sp, stp, wu, 2000, world, rank, dist,
                                                   "cpu" if args.shared_gpu else "cuda")
            except Exception as exc:   # report, never fail the bench on a config leg
                multi_cfg[name] = {"value": None, "error": repr(exc)[:300]}

    st_launch = {k: v // Q for k, v in st.items()}   # one engine's launch (Q equal slices)
    if rank == 0:
        traffic, step_traffic, traffic_tag = pmc_traffic(S, N, Q)
        # Roofline kernel: the launch with the largest share of the timed step (engine 0's HIP
        # events in the timed region).  Its achieved rate comes from the isolated leg (engine 0
        # alone after the timed region, HIP events on its stream; with Q = 1 the timed region is
        # that already): in the timed region the two engines' launches interleave on the chip and
        # an event duration includes the other engine's share.  k_apply, the HBM-heaviest launch,
        # is reported beside it.
        ref_ms, ref_st = (iso_ms, st_iso) if iso_ms else (phase_ms, st_launch)
        slots_launch = (S // Q) * cap
        dom = max(phase_ms, key=lambda p: phase_ms[p])
        dom_ms = ref_ms[dom]
        b = kernel_bytes(dom, ref_st, slots_launch)
        achieved = b / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0

        def kline(p, t_ms, stc):
            alg = kernel_bytes(p, stc, slots_launch)
            k = traffic.get(PHASE_KERNEL[p], {})
            hbm = k.get("hbm_bytes_per_launch")
            gbs = alg / (t_ms * 1e-3) / 1e9 if t_ms > 0 else 0.0
            line = {"ms": t_ms, "alg_bytes": alg, "gbs": gbs,
                    "frac": gbs / HBM_PEAK_GBS,
                    "pmc_bytes": hbm,
                    "pmc_over_alg": (hbm / alg) if hbm and alg else None,
                    "rocprof_avg_us": k.get("avg_us_isolated" if ref_ms is iso_ms
                                            else "avg_us_timed")}
            if line["frac"] > 1.0:   # never a fraction above the peak: operands from on-die cache
                line.update(frac=None, bound="cache",
                            note="algorithmic bytes over the launch exceed the HBM peak: reads "
                                 "served from L2 / MALL")
            return line
        per_kernel = {p: kline(p, ref_ms[p], ref_st) for p in PHASES}
        overlapped = {p: {"ms": phase_ms[p],
                          "gbs": (kernel_bytes(p, st_launch, slots_launch) / (phase_ms[p] * 1e-3)
                                  / 1e9 if phase_ms[p] > 0 else 0.0)} for p in PHASES}
        # implemented minimum: what this build's six launches must move per update (the
        # per-kernel figures above, summed, over the streams); SURVEY §8(d)'s canonical figure
        # charges a dense N x M cost matrix and a 576-B Kalman state, neither of which exists here
        impl_bytes = sum(kernel_bytes(p, st, S * cap) for p in PHASES) / S
        pcie = (None if args.no_pcie else
                pcie_inclusive(frame_of, S, N, local_rank, first=min(PRE, FT - 8),
                               engines=args.pcie_engines))
        if pcie is not None and not args.no_pcie_pinned:
            pp = pcie_inclusive(frame_of, S, N, local_rank, first=min(PRE, FT - 8),
                                engines=args.pcie_engines, pinned=True)
            pcie["pinned"] = {k: pp[k] for k in ("value", "ms_per_step", "ms_per_step_all")}
            pcie["pinned"]["note"] = pp["note"]
        if pcie is not None:
            # 16 timed frames: the loop's fill and drain (two frames' latency not overlapped) are
            # charged to fewer frames at 8 (tools/pipe_frames_ab.sh, gpurun_out/r6w: 711 k at 8,
            # 756 k at 16, page-locked)
            PF = min(16, FT)
            pf0 = min(PRE, FT - PF)
            pcie["pipelined"] = pcie_pipelined(frame_of, S, N, local_rank, first=pf0, frames=PF)
            if not args.no_pcie_pinned:
                pcie["pipelined"]["pinned"] = pcie_pipelined(frame_of, S, N, local_rank,
                                                             first=pf0, frames=PF, pinned=True)
                pcie["pipelined"]["pinned_f32"] = pcie_pipelined(
                    frame_of, S, N, local_rank, first=pf0, frames=PF, pinned=True, f32=True)
        dropin = None if args.no_dropin else dropin_leg(N, 60, args.seed, f"cuda:{local_rank}")
        configs = None if args.no_configs else configs_leg(None if world == 1 else ["C2", "C3"])
        if multi_cfg:
            configs = dict(configs or {}, **multi_cfg)
        cpu = None if args.no_cpu_baseline else cpu_baseline(N, args.cpu_frames, args.seed)
        if dropin is not None and cpu and cpu.get("value"):
            dropin["vs_cpu_1core"] = dropin["value"] / cpu["value"]
        dk = traffic.get(PHASE_KERNEL[dom], {})
        line = {
            "metric": "tracker.update() calls/sec @ 1024 tracks×1024 dets; 1/2/4/8 MI355X",
            "value": value, "unit": "calls/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"bytetrack {N}x{N}, {S} streams/GPU, inputs resident in HBM",
                       "tracker": "bytetrack", "tracks": N, "dets": N, "streams_per_gpu": S,
                       "queues_per_gpu": Q, "parallelism": f"stream-sharded x{world}",
                       "untimed_frames": PRE, "preroll": args.preroll,
                       "timed_frames": f"{PRE + 1}..{F}",
                       "per_stream_last_frame": {
                           "pool": st["pool"] / S, "tracked": st["tracked"] / S,
                           "lost": st["lost"] / S, "births": st["births"] / S,
                           "out_rows": st["out"] / S},
                       "value_is": "device-resident: frames staged in HBM before the timed "
                                   "region, output rows left in HBM; the host-buffer rate "
                                   "(dets in, rows out over PCIe every call) is pcie_inclusive"},
            "roofline": {"bound": "hbm", "kernel": PHASE_KERNEL[dom], "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": dk.get("hbm_bytes_per_launch"),
                         "traffic_over_alg": (dk["hbm_bytes_per_launch"] / b
                                              if dk.get("hbm_bytes_per_launch") else None),
                         "traffic_source": (f"profiles/{traffic_tag}_summary.json (rocprofv3 "
                                            f"{PHASE_KERNEL[dom]}: FETCH_SIZE x2 + WRITE_SIZE, "
                                            "isolated launches)" if dk else None),
                         "algorithmic_bytes_per_launch": b, "avg_launch_ms": dom_ms,
                         "rocprof_avg_launch_ms": (dk.get("avg_us_isolated") / 1e3
                                                   if dk.get("avg_us_isolated") else None),
                         "launch_streams": S // Q,
                         "timing": ("isolated leg: engine 0 alone for the frames after the timed "
                                    "region, HIP events on its stream" if iso_ms else
                                    "timed region, HIP events on the engine stream"),
                         "isolated_frames": ISO,
                         # every kernel of every engine: measured HBM bytes per step / step time
                         "chip_gbs": (step_traffic / (ms_per_step * 1e-3) / 1e9
                                      if step_traffic else None),
                         "beside": {p: dict(per_kernel[p], timed_ms=phase_ms[p],
                                            timed_share=(phase_ms[p] / ms_per_step
                                                         if ms_per_step > 0 else None))
                                    for p in ("apply", "s1_edges", "finish") if p != dom},
                         "selection": "the launch with the largest timed share (engine 0's HIP "
                                      "events in the timed window); its achieved rate from the "
                                      "isolated leg",
                         "timed_share": {p: (phase_ms[p] / ms_per_step if ms_per_step > 0
                                             else None) for p in PHASES},
                         "timed_share_note": "each kernel's average launch in the timed region "
                                             "(engine 0's HIP events; the engines' launches "
                                             "overlap, so the shares sum to more than 1) / "
                                             "ms_per_step",
                         "overlapped": (None if Q == 1 else {
                             "avg_launch_ms": phase_ms[dom],
                             "frac": (kernel_bytes(dom, st_launch, slots_launch)
                                      / (phase_ms[dom] * 1e-3) / 1e9
                                      / HBM_PEAK_GBS if phase_ms[dom] > 0 else None),
                             "note": f"{Q} engines of {S // Q} streams on {Q} HIP streams in the "
                                     "timed region: each launch overlaps the other engines' "
                                     "kernels, so its event duration includes their share"})},
            "pcie_inclusive": pcie,
            "cpu_baseline": cpu,
            "dropin": dropin,
            "configs": configs,
            "per_kernel": per_kernel,
            "per_kernel_overlapped": overlapped,
            "frame_counts": st,
            "busiest_kernel": dom,
            "kernel_bytes_note": "per_kernel.alg_bytes: bench.kernel_bytes (every array element a "
                                 "launch must read or write once, from the frame's counts); "
                                 "pmc_bytes: rocprofv3 counters of the same kernel "
                                 "(profiles/roofline_traffic.json); the ratio above 1 is line "
                                 "granularity and whole-line writes",
            "algorithmic_bytes_per_update": impl_bytes,
            "algorithmic_bytes_note": "implemented minimum (sum of the six launches' algorithmic "
                                      "bytes / streams); SURVEY §8(d)'s canonical figure "
                                      "(dense_upper_bound) charges a dense 16*N*M cost matrix "
                                      "and a 576-B Kalman state that this build never forms",
            "dense_upper_bound_bytes_per_update": algorithmic_bytes(N, N),
            "stage_seconds": round(gen_s, 1),
            "host_peak_rss_mb_by_rank": rss,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
