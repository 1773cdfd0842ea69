"""yolo_tracking_amd — MI355X-native tracker.update() hot path with BoxMOT's plugin surface.

    from yolo_tracking_amd import create_tracker, get_tracker_config
    tracker = create_tracker('bytetrack', get_tracker_config('bytetrack'), None, 0, False, False)
    tracks = tracker.update(dets, img)     # (K, 8) [x1, y1, x2, y2, id, conf, cls, det_ind]

Reference surface: boxmot/__init__.py:5-18.  The arithmetic runs in the gfx950 library
`libyta.so` (C ABI: include/yolo_tracking_amd.h); there is no CPU fallback.
"""
__version__ = "10.0.51+mi355x.1"

from .tracker_zoo import create_tracker, get_tracker_config  # noqa: E402
from .trackers.bytetrack import BYTETracker, ByteTrackEngine  # noqa: E402
from .trackers.botsort import BoTSORT, BoTSORTEngine  # noqa: E402
from .trackers.ocsort import OCSort, OCSortEngine  # noqa: E402
from .trackers.deepocsort import DeepOCSort, DeepOCSortEngine  # noqa: E402
from .trackers.hybridsort import HybridSORT, HybridSortEngine  # noqa: E402
from .postprocessing.gsi import gsi  # noqa: E402

TRACKERS = ["bytetrack", "botsort", "strongsort", "ocsort", "deepocsort", "hybridsort"]

__all__ = ("__version__", "BYTETracker", "ByteTrackEngine", "BoTSORT", "BoTSORTEngine", "OCSort",
           "OCSortEngine", "DeepOCSort", "DeepOCSortEngine", "HybridSORT", "HybridSortEngine",
           "create_tracker",
           "get_tracker_config", "gsi", "TRACKERS")
