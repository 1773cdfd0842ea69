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
    if tracker_type == "botsort":
        from .trackers.botsort import BoTSORT
        # reid_weights names the reference's ReID model (outside the hot path); an object with
        # get_features(xyxys, img) passed in its place is used as the feature producer
        reid = reid_weights if hasattr(reid_weights, "get_features") else None
        return BoTSORT(reid_weights, device, half, track_high_thresh=cfg.track_high_thresh,
                       track_low_thresh=cfg.track_low_thresh,
                       new_track_thresh=cfg.new_track_thresh, track_buffer=cfg.track_buffer,
                       match_thresh=cfg.match_thresh, proximity_thresh=cfg.proximity_thresh,
                       appearance_thresh=cfg.appearance_thresh, cmc_method=cfg.cmc_method,
                       frame_rate=cfg.frame_rate, reid=reid)
    if tracker_type == "ocsort":
        from .trackers.ocsort import OCSort
        return OCSort(per_class, det_thresh=cfg.det_thresh, max_age=cfg.max_age,
                      min_hits=cfg.min_hits, asso_threshold=cfg.iou_thresh, delta_t=cfg.delta_t,
                      asso_func=cfg.asso_func, inertia=cfg.inertia, use_byte=cfg.use_byte,
                      device=device)
    if tracker_type == "deepocsort":
        from .trackers.deepocsort import DeepOCSort
        reid = reid_weights if hasattr(reid_weights, "get_features") else None
        return DeepOCSort(reid_weights, device, half, per_class, det_thresh=cfg.det_thresh,
                          max_age=cfg.max_age, min_hits=cfg.min_hits,
                          iou_threshold=cfg.iou_thresh, delta_t=cfg.delta_t,
                          asso_func=cfg.asso_func, inertia=cfg.inertia, reid=reid)
    if tracker_type == "hybridsort":
        from .trackers.hybridsort import HybridSORT
        reid = reid_weights if hasattr(reid_weights, "get_features") else None
        return HybridSORT(reid_weights, device, half, det_thresh=cfg.det_thresh,
                          max_age=cfg.max_age, min_hits=cfg.min_hits,
                          iou_threshold=cfg.iou_thresh, delta_t=cfg.delta_t,
                          asso_func=cfg.asso_func, inertia=cfg.inertia, reid=reid)
    if tracker_type == "strongsort":
        raise NotImplementedError(
            f"{tracker_type}: not yet on the MI355X path in this build; see DESIGN.md")
    print("No such tracker")
    exit()
