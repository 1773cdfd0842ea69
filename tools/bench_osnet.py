"""ReID producer end to end on the MI355X: crops of S camera streams x M
detections (1920x1080 BGR, one yta_reid_preprocess_device launch) + the OSNet forward
(appearance/osnet.py: folded BatchNorms, channels-last, batched branches; random weights of the
named variant) + global normalisation, features left on the device.  Reports crops/s for the
network alone and for the whole get_features path, float32 and float16.  Prints JSON lines."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="osnet_x0_25")
    ap.add_argument("--crops", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from yolo_tracking_amd.appearance import ReIDDetectMultiBackend
    from yolo_tracking_amd.appearance.osnet import OSNetReID
    rng = np.random.default_rng(0)
    H, W, n = 1080, 1920, args.crops
    img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    wh = rng.uniform(48, 192, (n, 2))
    xy = rng.uniform(0, 1, (n, 2)) * [W - 200, H - 200]
    boxes = np.concatenate([xy, xy + wh], 1)
    for half, chunk, hip, cl in ((False, 1024, True, False), (True, 1024, True, False),
                                 (False, 256, True, False), (True, 256, True, False),
                                 (False, 1024, False, True), (True, 1024, False, True),
                                 (True, 1024, False, False)):
        net = OSNetReID(args.variant, None, device="cuda:0", half=half, chunk=chunk,
                        channels_last=cl, hip=hip)
        reid = ReIDDetectMultiBackend(None, device=0, fp16=half, model=net)
        crops = reid.preprocess(boxes, img)
        if half:
            crops = crops.half()
        for _ in range(3):
            net(crops)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            net(crops)
        e1.record()
        torch.cuda.synchronize()
        net_ms = e0.elapsed_time(e1) / args.steps
        reid.get_features(boxes, img)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            reid.get_features(boxes, img)
        e2e_ms = 1000 * (time.perf_counter() - t0) / args.steps
        print(json.dumps({"metric": "OSNet ReID crops/s", "variant": args.variant,
                          "dtype": "f16" if half else "f32", "crops": n, "chunk": chunk,
                          "layout": "nhwc" if cl else "nchw", "hip_blocks": hip,
                          "network_ms": net_ms, "network_crops_per_s": n / (net_ms * 1e-3),
                          "get_features_ms": e2e_ms,
                          "get_features_crops_per_s": n / (e2e_ms * 1e-3),
                          "note": "get_features: host image -> device, crops, network, global "
                                  "norm, features back to the host (synchronous)"}))


if __name__ == "__main__":
    main()
