#!/usr/bin/env python3
"""Per-config throughput of the other trackers (BASELINE.json configs 2 and 3).

    python tools/bench_tracker.py --tracker ocsort  [--n 256]  [--streams 1] [--steps 50]
    python tools/bench_tracker.py --tracker botsort [--n 1024] [--dim 512] [--streams 1]
    python tools/bench_tracker.py --tracker deepocsort [--n 2048] [--dim 512] [--streams 1]
    python tools/bench_tracker.py --tracker hybridsort [--n 4096] [--dim 512] [--streams 8]

A step = one update() frame of every stream (SURVEY.md §8(d) synthetic streams; OCSORT with
ocsort.yaml parameters and no low-confidence detections, BoT-SORT with botsort.yaml parameters
and D-dim float32 embeddings through the get_features convention), inputs staged in HBM, the
engine's device-buffer entry point, K timed frames bracketed by device syncs.  The CPU baseline
is the oracle restatement of the same tracker on one core over a bounded sample of the stream.
bench.py (the driver's contract) measures the ByteTrack headline; this tool is for DESIGN.md.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

OCSORT_YAML = dict(det_thresh=0.0, max_age=30, min_hits=1, asso_threshold=0.3, delta_t=3,
                   asso_func="giou", inertia=0.2, use_byte=False)
BOTSORT_YAML = dict(track_high_thresh=0.33824964456239337, track_low_thresh=0.1,
                    new_track_thresh=0.21144301345190655, track_buffer=60,
                    match_thresh=0.22734550911325851, proximity_thresh=0.5945380911899254,
                    appearance_thresh=0.4818211117541298, frame_rate=30)
DEEPOCSORT_YAML = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
                       asso_func="giou", inertia=0.2)          # create_tracker's arguments
HYBRIDSORT_YAML = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
                       asso_func="giou", inertia=0.2)
CMC_AFFINE = [[1.0, 1e-3, 0.5], [-1e-3, 1.0, -0.3]]
DEFAULT_N = {"ocsort": 256, "botsort": 1024, "deepocsort": 2048, "hybridsort": 4096}


def reid_rows(dets, embs, thr):
    f = embs[dets[:, 4] > thr]
    return (f / np.linalg.norm(f)).astype(np.float32) if len(f) else f


def cpu_leg(code, timeout=900):
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    try:
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           timeout=timeout)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as exc:
        return {"error": str(exc)}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--tracker", choices=["ocsort", "botsort", "deepocsort", "hybridsort"],
                   required=True)
    p.add_argument("--n", type=int, default=None)
    p.add_argument("--dim", type=int, default=512)
    p.add_argument("--streams", type=int, default=1)
    p.add_argument("--queues", type=int, default=None,
                   help="deepocsort / hybridsort: Q engines of streams/Q streams, each on its own "
                        "HIP stream, so one engine's one-block-per-stream solve overlaps another's "
                        "chip-wide GEMM (default 2 for an even stream count, else 1; "
                        "profiles/r03zf_queues_sweep.txt)")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--cpu-frames", type=int, default=None)
    p.add_argument("--seed", type=int, default=2000)
    return p.parse_args(argv)


def cpu_code(args, N, D, cf):
    """The oracle leg's script (one stream, one thread, frames 2..cf+1), or None."""
    oc = args.tracker == "ocsort"
    if cf == 0:
        return None
    if args.tracker == "deepocsort":
        return ("import sys,time,json; sys.path.insert(0,%r)\n"
                "import numpy as np\n"
                "from oracle.deepocsort import DeepOCSortOracle\n"
                "from yolo_tracking_amd.synth import make_frames, SyntheticStream\n"
                "fr=make_frames(%d,%d,%d,emb_dim=%d,low_conf_frac=0.0)\n"
                "sh=SyntheticStream(%d,%d,emb_dim=%d,low_conf_frac=0.0).img_shape\n"
                "w=np.array(%r)\n"
                "t=DeepOCSortOracle(**%r); t.update(fr[0][0],sh,fr[0][1]/np.linalg.norm(fr[0][1]),w)\n"
                "t0=time.perf_counter()\n"
                "for d,e in fr[1:]: t.update(d,sh,e/np.linalg.norm(e),w)\n"
                "print(json.dumps({'frames':len(fr)-1,'seconds':time.perf_counter()-t0}))\n"
                % (REPO, N, cf + 1, args.seed, D, N, args.seed, D, CMC_AFFINE, DEEPOCSORT_YAML))
    if args.tracker == "hybridsort":
        return ("import sys,time,json; sys.path.insert(0,%r)\n"
                "import numpy as np\n"
                "from oracle.hybridsort import HybridSortOracle\n"
                "from yolo_tracking_amd.synth import make_frames\n"
                "fr=make_frames(%d,%d,%d,emb_dim=%d,low_conf_frac=0.0)\n"
                "t=HybridSortOracle(**%r); t.update(fr[0][0],fr[0][1]/np.linalg.norm(fr[0][1]))\n"
                "t0=time.perf_counter()\n"
                "for d,e in fr[1:]: t.update(d,e/np.linalg.norm(e))\n"
                "print(json.dumps({'frames':len(fr)-1,'seconds':time.perf_counter()-t0}))\n"
                % (REPO, N, cf + 1, args.seed, D, HYBRIDSORT_YAML))
    if oc:
        return ("import sys,time,json; sys.path.insert(0,%r)\n"
                "from oracle.ocsort import OCSortOracle\n"
                "from yolo_tracking_amd.synth import make_frames, SyntheticStream\n"
                "fr=[d for d,_ in make_frames(%d,%d,%d,low_conf_frac=0.0)]\n"
                "sh=SyntheticStream(%d,%d,low_conf_frac=0.0).img_shape\n"
                "t=OCSortOracle(**%r); t.update(fr[0],sh)\n"
                "t0=time.perf_counter()\n"
                "for d in fr[1:]: t.update(d,sh)\n"
                "print(json.dumps({'frames':len(fr)-1,'seconds':time.perf_counter()-t0}))\n"
                % (REPO, N, cf + 1, args.seed, N, args.seed, OCSORT_YAML))
    return ("import sys,time,json; sys.path.insert(0,%r)\n"
            "import numpy as np\n"
            "from oracle.botsort import BoTSORTOracle\n"
            "from yolo_tracking_amd.synth import make_frames\n"
            "fr=make_frames(%d,%d,%d,emb_dim=%d)\n"
            "kw=%r\n"
            "def rows(d,e):\n"
            "    f=e[d[:,4]>kw['track_high_thresh']]; return f/np.linalg.norm(f)\n"
            "t=BoTSORTOracle(**kw); t.update(fr[0][0],rows(*fr[0]))\n"
            "t0=time.perf_counter()\n"
            "for d,e in fr[1:]: t.update(d,rows(d,e))\n"
            "print(json.dumps({'frames':len(fr)-1,'seconds':time.perf_counter()-t0}))\n"
            % (REPO, N, cf + 1, args.seed, D, BOTSORT_YAML))


def default_cpu_frames(args):
    oc = args.tracker == "ocsort"
    fam = args.tracker in ("deepocsort", "hybridsort")
    return args.cpu_frames if args.cpu_frames is not None else (30 if oc else (2 if fam else 6))


def start_cpu_leg(args):
    """The oracle leg as a background process (bench.py runs it beside the GPU legs)."""
    N = args.n or DEFAULT_N[args.tracker]
    D = 0 if args.tracker == "ocsort" else args.dim
    cf = default_cpu_frames(args)
    code = cpu_code(args, N, D, cf)
    if code is None:
        return None, cf
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    return subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True), cf


def finish_cpu_leg(args, proc, cf, timeout=900):
    N = args.n or DEFAULT_N[args.tracker]
    if proc is None:
        res = {"error": "skipped (--cpu-frames 0)"}
    else:
        try:
            out, _ = proc.communicate(timeout=timeout)
            res = json.loads(out.strip().splitlines()[-1])
        except Exception as exc:
            res = {"error": str(exc)}
    return ({"value": res["frames"] / res["seconds"], "unit": "calls/s", "cores": 1, "kind": "port",
             "sample": f"oracle {args.tracker} 1 stream {N}x{N}, frames 2..{cf + 1} of seed "
                       f"{args.seed}, {res['seconds']:.1f} s, 1 thread"}
            if "frames" in res else {"value": None, "sample": res.get("error")})


def run(args, cpu=None, seeds=None, barrier=None):
    """One config on the GPU -> its JSON line.  cpu: a (process, frames) pair from start_cpu_leg
    to collect for the line's cpu_baseline (None: run the CPU leg here, after the GPU legs;
    (None, 0): no CPU leg).  seeds: the streams' generator seeds (default seed + s; bench.py's
    multi-GPU legs pass stream s's global seed, streams sharded s mod G over the ranks).
    barrier: called on both sides of the timed region after the device syncs (bench.py: the
    ranks' barrier, so the slowest rank's elapsed time is the job's)."""
    import torch
    from yolo_tracking_amd import _lib
    from yolo_tracking_amd.synth import SyntheticStream, make_frames
    S = args.streams
    if args.queues is None:
        args.queues = 2 if S >= 2 and S % 2 == 0 else 1
    F = args.warmup + args.steps
    oc = args.tracker == "ocsort"
    fam = args.tracker in ("deepocsort", "hybridsort")
    N = args.n or DEFAULT_N[args.tracker]
    D = 0 if oc else args.dim
    kw_stream = dict(low_conf_frac=0.0) if oc else dict(emb_dim=D)
    if fam:
        kw_stream["low_conf_frac"] = 0.0
    if seeds is None:
        seeds = [args.seed + s for s in range(S)]
    assert len(seeds) == S
    streams = [make_frames(N, F, seeds[s], **kw_stream) for s in range(S)]
    dets = np.stack([np.concatenate([streams[s][f][0] for s in range(S)]) for f in range(F)])
    off = np.array([[sum(len(streams[q][f][0]) for q in range(s)) for s in range(S + 1)]
                    for f in range(F)], dtype=np.int32)
    d_dets = torch.from_numpy(dets).cuda()
    d_off = torch.from_numpy(off).cuda()
    row_bytes = dets.shape[1] * 6 * 8
    if oc:
        from yolo_tracking_amd.trackers.ocsort import OCSortEngine
        eng = OCSortEngine(S, **OCSORT_YAML, track_capacity=2 * N, max_dets=N)
        shape = SyntheticStream(N, args.seed, **kw_stream).img_shape
        d_wh = torch.tensor([[shape[1], shape[0]]] * S, dtype=torch.int32).cuda()
        cap, _ = eng.capacity()
        d_out = torch.empty((S * cap, 8), dtype=torch.float64, device="cuda")
        fn, sync = eng.lib.yta_ocsort_update_device, eng.lib.yta_ocsort_sync

        def step(f):
            _lib.check(fn(eng.handle, ctypes.c_void_p(d_dets.data_ptr() + f * row_bytes),
                          ctypes.c_void_p(d_off.data_ptr() + f * (S + 1) * 4),
                          ctypes.c_void_p(d_wh.data_ptr()), ctypes.c_void_p(d_out.data_ptr()),
                          None))
    elif fam:
        # get_features rows of every detection (all rows kept at det_thresh 0), global norm per
        # stream-frame (reid_multibackend.py:310)
        feats = np.zeros((F, dets.shape[1], D), np.float32)
        for f in range(F):
            r0 = 0
            for s in range(S):
                d, e = streams[s][f]
                feats[f, r0:r0 + len(d)] = e / np.linalg.norm(e)
                r0 += len(d)
        d_feat = torch.from_numpy(feats).cuda()
        del feats
        feat_bytes = dets.shape[1] * D * 4
        Q = max(1, args.queues)
        assert S % Q == 0, "--streams must be a multiple of --queues"
        Sq = S // Q
        engines, calls = [], []
        if args.tracker == "deepocsort":
            from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine
            shape = SyntheticStream(N, args.seed, **kw_stream).img_shape
            d_warp = torch.tensor([CMC_AFFINE] * S, dtype=torch.float64).cuda()
            d_wh = torch.tensor([[shape[1], shape[0]]] * S, dtype=torch.int32).cuda()
        else:
            from yolo_tracking_amd.trackers.hybridsort import HybridSortEngine
        for q in range(Q):
            # engine q: streams q*Sq .. (q+1)*Sq - 1, detection offsets rebased to its first row
            base = off[:, q * Sq].astype(np.int64)
            d_offq = torch.from_numpy(
                np.ascontiguousarray(off[:, q * Sq:(q + 1) * Sq + 1] - base[:, None]).astype(np.int32)).cuda()
            if args.tracker == "deepocsort":
                e = DeepOCSortEngine(Sq, feat_dim=D, **DEEPOCSORT_YAML, track_capacity=2 * N,
                                     max_dets=N)
                fn, sync1 = e.lib.yta_deepocsort_update_device, e.lib.yta_deepocsort_sync
            else:
                e = HybridSortEngine(Sq, feat_dim=D, **HYBRIDSORT_YAML, track_capacity=2 * N,
                                     max_dets=N)
                fn, sync1 = e.lib.yta_hybridsort_update_device, e.lib.yta_hybridsort_sync
            cap, _ = e.capacity()
            d_out = torch.empty((Sq * cap, 8), dtype=torch.float64, device="cuda")
            engines.append(e)
            calls.append((fn, d_offq, base, q, d_out))
        eng = engines[0]

        class _AllSync:   # sync(handle) over every engine (the handle argument is ignored)
            def __call__(self, _handle):
                for e_ in engines:
                    rc = sync1(e_.handle)
                    if rc:
                        return rc
                return 0
        sync = _AllSync()

        def step(f):
            for (fn_, d_offq, base, q, d_out), e_ in zip(calls, engines):
                r0 = int(base[f])
                pd = ctypes.c_void_p(d_dets.data_ptr() + f * row_bytes + r0 * 48)
                po = ctypes.c_void_p(d_offq.data_ptr() + f * (Sq + 1) * 4)
                pf = ctypes.c_void_p(d_feat.data_ptr() + f * feat_bytes + r0 * D * 4)
                if args.tracker == "deepocsort":
                    _lib.check(fn_(e_.handle, pd, po, pf,
                                   ctypes.c_void_p(d_warp.data_ptr() + q * Sq * 6 * 8),
                                   ctypes.c_void_p(d_wh.data_ptr() + q * Sq * 2 * 4),
                                   ctypes.c_void_p(d_out.data_ptr()), None))
                else:
                    _lib.check(fn_(e_.handle, pd, po, pf, ctypes.c_void_p(d_out.data_ptr()), None))
    else:
        from yolo_tracking_amd.trackers.botsort import BoTSORTEngine
        eng = BoTSORTEngine(S, feat_dim=D, **BOTSORT_YAML, track_capacity=2 * N, max_dets=N)
        # ReID rows aligned with the detections (the high rows carry get_features' output)
        feats = np.zeros((F, dets.shape[1], D), np.float32)
        for f in range(F):
            r0 = 0
            for s in range(S):
                d, e = streams[s][f]
                hi = d[:, 4] > BOTSORT_YAML["track_high_thresh"]
                blk = np.zeros((len(d), D), np.float32)
                blk[hi] = reid_rows(d, e, BOTSORT_YAML["track_high_thresh"])
                feats[f, r0:r0 + len(d)] = blk
                r0 += len(d)
        d_feat = torch.from_numpy(feats).cuda()
        feat_bytes = dets.shape[1] * D * 4
        cap, _ = eng.capacity()
        d_out = torch.empty((S * cap, 8), dtype=torch.float64, device="cuda")
        fn, sync = eng.lib.yta_botsort_update_device, eng.lib.yta_bytetrack_sync

        def step(f):
            _lib.check(fn(eng.handle, ctypes.c_void_p(d_dets.data_ptr() + f * row_bytes),
                          ctypes.c_void_p(d_off.data_ptr() + f * (S + 1) * 4),
                          ctypes.c_void_p(d_feat.data_ptr() + f * feat_bytes), None,
                          ctypes.c_void_p(d_out.data_ptr()), None))
    for f in range(args.warmup):
        step(f)
    _lib.check(sync(eng.handle))
    torch.cuda.synchronize()
    stamps = os.environ.get("YTA_HS_STAMPS") and args.tracker == "hybridsort"
    if stamps:   # diagnostic library: k_hs_lap's solver phases over the timed frames
        eng.lib.yta_hs_debug_stamps_reset()
    if barrier is not None:
        barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(args.warmup, F):
        step(f)
    _lib.check(sync(eng.handle))
    torch.cuda.synchronize()
    if barrier is not None:
        barrier()
    el = time.perf_counter() - t0
    value = S * args.steps / el
    if stamps:
        st = np.zeros(128, np.uint64)
        fnst = eng.lib.yta_hs_debug_stamps
        fnst.argtypes = [ctypes.c_void_p]
        _lib.check(fnst(st.ctypes.data))
        print(f"k_hs_lap (block 0, {args.steps} frames): free rows {int(st[100])}, steps "
              f"{int(st[101])}, scan {int(st[102]) / 100:.0f} us, reduce {int(st[103]) / 100:.0f} us, "
              f"bidding rounds {int(st[106])} ({int(st[107]) / 100:.0f} us)",
              file=sys.stderr)
        names = ["first round", "lists", "updates", "OCR round", "misses", "births", "outputs"]
        ph = [f"{nm} {(int(st[41 + k]) - int(st[40 + k])) / 100:.1f}" for k, nm in enumerate(names)
              if st[41 + k] and st[40 + k] and st[41 + k] >= st[40 + k]]
        print("k_hs_assoc (block 0, last frame, us): " + ", ".join(ph), file=sys.stderr)
        if st[48] and st[43] and st[44] >= st[48] >= st[43]:
            print(f"  OCR round: matrix {(int(st[48]) - int(st[43])) / 100:.1f} us, solve "
                  f"{(int(st[44]) - int(st[48])) / 100:.1f} us ({int(st[49])} x {int(st[50])}: {int(st[51])} free "
                  f"rows, {int(st[52])} search steps)", file=sys.stderr)
            if st[104] >= st[48] and st[105] >= st[104]:   # lap_rect_body's stamps, last call
                print(f"  OCR solve: pre-pass + claims {(int(st[104]) - int(st[48])) / 100:.1f} us, "
                      f"searches {(int(st[105]) - int(st[104])) / 100:.1f} us", file=sys.stderr)
    stats = eng.stats()
    if fam and len(engines) > 1:   # summed over the engines: the same totals as one engine of S
        for e_ in engines[1:]:
            for k, v in e_.stats().items():
                if isinstance(v, (int, float)) and isinstance(stats.get(k), (int, float)):
                    stats[k] += v
    # CPU leg: the oracle on stream 0, 1 thread, bounded sample
    if cpu is None:
        cpu = start_cpu_leg(args)
    cpu = finish_cpu_leg(args, *cpu)
    line = {"metric": f"{args.tracker} tracker.update() calls/sec @ {N} tracks x {N} dets",
            "value": value, "unit": "calls/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000 * el / args.steps,
            "higher_is_better": True, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{args.tracker} {N}x{N}" + (f" D={D}" if D else "")
                                   + f", {S} streams, inputs resident in HBM",
                       "streams": S, "queues": max(1, args.queues) if fam else 1},
            "cpu_baseline": cpu, "frame_counts": stats, "elapsed_s": el,
            "stream_seeds": list(seeds)}
    return line


def main():
    print(json.dumps(run(parse())))


if __name__ == "__main__":
    main()
