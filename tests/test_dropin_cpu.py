"""CPU: examples/track.py's boxmot surface resolves through the alias package (reference
examples/track.py:9-12, :15-16, :37-41; boxmot/utils/checks.py:10-35; tracker_zoo.py:20-22)."""
import sys

import yaml

import dropin


def test_track_py_imports_and_config_paths():
    ns = dropin.track_py_namespace()
    import boxmot
    import yolo_tracking_amd
    assert ns["TRACKERS"] == ["bytetrack", "botsort", "strongsort", "ocsort", "deepocsort",
                              "hybridsort"]
    # the alias hands out the package's own objects (shared ID counters, one loaded library)
    assert ns["create_tracker"] is yolo_tracking_amd.create_tracker
    assert sys.modules["boxmot.tracker_zoo"] is sys.modules["yolo_tracking_amd.tracker_zoo"]
    assert boxmot.BYTETracker is yolo_tracking_amd.BYTETracker
    from boxmot.trackers.bytetrack.byte_tracker import BYTETracker
    from boxmot.trackers.ocsort.ocsort import OCSort
    from boxmot.postprocessing.gsi import gsi  # noqa: F401
    assert BYTETracker is yolo_tracking_amd.BYTETracker and OCSort is yolo_tracking_amd.OCSort
    # requirement check: reported, never installed
    assert ns["__tr"].missing == [
        "ultralytics @ git+https://github.com/mikel-brostrom/ultralytics.git"]
    assert ns["TestRequirements"]().check_requirements() == []
    # track.py:37-41 builds the YAML path from ROOT; get_tracker_config points at the same files
    keys = {"bytetrack": ["track_thresh", "match_thresh", "track_buffer", "frame_rate"],
            "botsort": ["track_high_thresh", "track_low_thresh", "new_track_thresh",
                        "track_buffer", "match_thresh", "proximity_thresh", "appearance_thresh",
                        "cmc_method", "frame_rate"],
            "ocsort": ["det_thresh", "max_age", "min_hits", "iou_thresh", "delta_t", "asso_func",
                       "inertia", "use_byte"],
            "deepocsort": ["det_thresh", "max_age", "min_hits", "iou_thresh", "delta_t",
                           "asso_func", "inertia"],
            "hybridsort": ["det_thresh", "max_age", "min_hits", "iou_thresh", "delta_t",
                           "asso_func", "inertia"],
            "strongsort": []}
    for m in ns["TRACKERS"]:
        p = dropin.tracking_config(ns, m)
        assert p.is_file(), p
        assert p == yolo_tracking_amd.get_tracker_config(m)
        cfg = yaml.safe_load(p.read_text())
        for k in keys[m]:
            assert k in cfg, (m, k)
    assert ns["WEIGHTS"] == ns["ROOT"] / "examples" / "weights"


def test_alias_leaves_native_package_untouched():
    """Importing boxmot must not replace yolo_tracking_amd's own submodule attributes with the
    alias-only namespaces (boxmot.trackers.bytetrack etc.)."""
    import importlib

    import boxmot  # noqa: F401
    import yolo_tracking_amd.motion
    import yolo_tracking_amd.trackers
    from yolo_tracking_amd.trackers import bytetrack, ocsort
    assert yolo_tracking_amd.trackers.bytetrack is bytetrack
    assert hasattr(yolo_tracking_amd.trackers.bytetrack, "ByteTrackEngine")
    m = importlib.import_module("yolo_tracking_amd.trackers.ocsort")
    assert m is ocsort and hasattr(m, "OCSort")
    assert not hasattr(yolo_tracking_amd.motion.cmc, "sof")
    # the reference paths still resolve, attribute access included
    import boxmot.trackers.bytetrack.byte_tracker as bt
    assert bt is bytetrack
    assert boxmot.trackers.bytetrack.byte_tracker.BYTETracker is bytetrack.BYTETracker
    assert boxmot.trackers.ocsort.ocsort.OCSort is ocsort.OCSort
    assert boxmot.motion.cmc.sof.SparseOptFlow is importlib.import_module(
        "yolo_tracking_amd.motion.sof").SparseOptFlow
    from boxmot.utils import ROOT  # noqa: F401
