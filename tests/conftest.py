import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")

# torch bundles its own libamdhip64; importing it before libyta.so is loaded makes the library bind
# to that same HIP runtime (one runtime per process).  Loading libyta.so first and torch later
# leaves torch on /opt/rocm's runtime, where it finds no GPU (tests/test_gpu_reid.py needs both).
try:
    import torch  # noqa: F401
except ImportError:   # pragma: no cover
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def mot_frames(g, key):
    """Rebuild per-frame detections of one MOT17-mini sequence from the golden fixture
    (det.txt rows frame,-1,left,top,w,h,conf -> [x1,y1,x2,y2,conf,0])."""
    import numpy as np
    q = g[f"{key}__det_milli"] / 1000.0
    fr = q[:, 0].astype(int)
    frames = []
    for f in range(1, fr.max() + 1):
        r = q[fr == f]
        d = np.zeros((len(r), 6))
        d[:, 0] = r[:, 1]
        d[:, 1] = r[:, 2]
        d[:, 2] = r[:, 1] + r[:, 3]
        d[:, 3] = r[:, 2] + r[:, 4]
        d[:, 4] = r[:, 5]
        frames.append(d)
    return frames
