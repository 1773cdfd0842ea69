"""create_tracker / get_tracker_config — the reference's plugin surface (boxmot/tracker_zoo.py:10-118).

Same signature, same YAML keys, same error behaviour (unknown tracker type prints and exits).
"""
from types import SimpleNamespace

import yaml

from .utils import BOXMOT


def get_tracker_config(tracker_type):
    """tracker_zoo.py:10-15."""
    return BOXMOT / "configs" / (tracker_type + ".yaml")


def create_tracker(tracker_type, tracker_config, reid_weights, device, half, per_class):
    """tracker_zoo.py:18-118."""
    with open(tracker_config, "r") as f:
        cfg = SimpleNamespace(**yaml.safe_load(f.read()))

    if tracker_type == "bytetrack":
        from .trackers.bytetrack import BYTETracker
        return BYTETracker(track_thresh=cfg.track_thresh, match_thresh=cfg.match_thresh,
                           track_buffer=cfg.track_buffer, frame_rate=cfg.frame_rate,
                           device=device)
    if tracker_type in ("ocsort", "botsort", "deepocsort", "hybridsort", "strongsort"):
        raise NotImplementedError(
            f"{tracker_type}: not yet on the MI355X path in this build (ByteTrack is); see DESIGN.md")
    print("No such tracker")
    exit()
