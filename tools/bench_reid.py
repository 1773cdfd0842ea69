"""ReID crop preprocessing throughput: S camera streams x M detections per frame,
one 1920x1080 BGR image per stream, boxes from the §8(d) generator scaled to the image; every crop
of every stream in one yta_reid_preprocess_device launch, images and boxes resident in HBM.
Roofline: HBM writes of the float32 / float16 NCHW crops (+ the crop source bytes, read once).
CPU leg: oracle/reid.py (the NumPy restatement of the reference's per-crop loop) on a bounded
sample.  Prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--dets", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--half", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=256)
    args = ap.parse_args()
    import torch
    from yolo_tracking_amd import _lib
    lib = _lib.load_library()
    d = torch.device("cuda", 0)
    S, M, H, W = args.streams, args.dets, 1080, 1920
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (S, H, W, 3), dtype=np.uint8)
    wh = rng.uniform(16, 64, (S, M, 2)) * 3          # 48..192 px boxes (people at 1080p)
    xy = rng.uniform(0, 1, (S, M, 2)) * [W - 200, H - 200]
    boxes = np.concatenate([xy, xy + wh], 2).reshape(-1, 4)
    n = S * M
    d_img = torch.from_numpy(imgs.reshape(-1)).to(d)
    d_off = torch.arange(S, dtype=torch.int64, device=d) * (H * W * 3)
    d_hw = torch.tensor([H, W] * S, dtype=torch.int32, device=d)
    d_box = torch.from_numpy(boxes).to(d)
    d_own = torch.arange(S, dtype=torch.int32, device=d).repeat_interleave(M)
    es = 2 if args.half else 4
    out = torch.empty((n, 3, 256, 128), dtype=torch.half if args.half else torch.float, device=d)
    st = torch.cuda.current_stream(d)

    def launch():
        _lib.check(lib.yta_reid_preprocess_device(
            ctypes.c_void_p(d_img.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
            ctypes.c_void_p(d_hw.data_ptr()), ctypes.c_void_p(d_box.data_ptr()),
            ctypes.c_void_p(d_own.data_ptr()), n, 256, 128, args.half,
            ctypes.c_void_p(out.data_ptr()), None, ctypes.c_void_p(st.cuda_stream)))

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.steps):
        launch()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    # practical write ceiling: the same output buffer filled by the runtime
    e0.record(st)
    for _ in range(args.steps):
        out.fill_(1.0)
    e1.record(st)
    torch.cuda.synchronize()
    fill_ms = e0.elapsed_time(e1) / args.steps
    # algorithmic bytes: output writes + source pixels of each crop (read once)
    wv = (boxes[:, 2].astype(int) - boxes[:, 0].astype(int))
    hv = (boxes[:, 3].astype(int) - boxes[:, 1].astype(int))
    src = float((wv * hv * 3).sum())
    wr = float(n * 3 * 256 * 128 * es)
    gbs = (wr + src + n * 36) / (ms * 1e-3) / 1e9
    # CPU leg: the oracle's per-crop loop (the reference's structure) on a sample of crops
    from oracle import reid as orr
    k = min(args.cpu_sample, M)
    t0 = time.perf_counter()
    orr.preprocess(boxes[:k], imgs[0])
    cpu_s = time.perf_counter() - t0
    print(json.dumps({"metric": "ReID crops preprocessed/s", "value": n / (ms * 1e-3),
                      "unit": "crops/s", "ms_per_launch": ms, "crops_per_launch": n,
                      "dtype": "f16" if args.half else "f32",
                      "config": {"workload": f"{S} streams x {M} dets, 1920x1080 BGR, 128x256 crops"},
                      "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s",
                                   "frac": gbs / 8000.0,
                                   "alg_bytes_per_launch": wr + src + n * 36,
                                   "fill_ceiling_gbs": wr / (fill_ms * 1e-3) / 1e9},
                      "cpu_baseline": {"value": k / cpu_s, "unit": "crops/s", "cores": 1,
                                       "kind": "port",
                                       "sample": f"oracle/reid.py preprocess, {k} crops of one image"}}))


if __name__ == "__main__":
    main()
