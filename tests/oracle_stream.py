"""Test helper (run as a subprocess, CPU only): one synthetic ByteTrack stream through the oracle.

    python tests/oracle_stream.py N FRAMES SEED OUT.npz

Regenerates the stream exactly as bench.py stages it (yolo_tracking_amd.synth.SyntheticStream(N,
SEED), frames 0..FRAMES-1) and runs oracle.bytetrack.ByteTrackOracle with the bench's parameters
(track_thresh 0.5, match_thresh 0.8, track_buffer 30, frame_rate 30); writes every frame's output
rows (concatenated), the per-frame row counts and the final ID counter.  Used by
tests/test_gpu_headline_shape.py to check sampled streams of the headline launch shape.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle.bytetrack import ByteTrackOracle  # noqa: E402
from yolo_tracking_amd.synth import SyntheticStream  # noqa: E402


def main(n, frames, seed, out):
    g = SyntheticStream(n, seed)
    o = ByteTrackOracle(track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30)
    rows, counts = [], []
    for _ in range(frames):
        d, _ = g.next_frame()
        r = np.asarray(o.update(d), dtype=np.float64).reshape(-1, 8)
        rows.append(r)
        counts.append(len(r))
    np.savez(out, rows=np.concatenate(rows) if rows else np.zeros((0, 8)),
             counts=np.asarray(counts, np.int64), next_id=np.int64(o.next_id))


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
