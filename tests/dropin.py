"""What examples/track.py does with `boxmot` (reference examples/track.py:9-12, :15-16, :25-57),
restated as data so the tests can run it through the alias package without importing
examples/* (which would pull the ultralytics fork and shell pip)."""
from types import SimpleNamespace

# examples/track.py:9-12, verbatim
IMPORT_LINES = """
from boxmot import TRACKERS
from boxmot.tracker_zoo import create_tracker
from boxmot.utils import ROOT, WEIGHTS
from boxmot.utils.checks import TestRequirements
"""


def track_py_namespace():
    """Execute track.py's four import lines and its import-time requirement check (:15-16) in a
    fresh namespace; returns the namespace."""
    ns = {}
    exec(compile(IMPORT_LINES, "examples/track.py", "exec"), ns)
    tr = ns["TestRequirements"]()
    tr.check_packages(("ultralytics @ git+https://github.com/mikel-brostrom/ultralytics.git", ))
    ns["__tr"] = tr
    return ns


def tracking_config(ns, method):
    """track.py:37-41."""
    return ns["ROOT"] / "boxmot" / "configs" / (method + ".yaml")


def on_predict_start(ns, predictor):
    """track.py:25-57 with the names bound by track_py_namespace()."""
    assert predictor.custom_args.tracking_method in ns["TRACKERS"]
    cfg = tracking_config(ns, predictor.custom_args.tracking_method)
    trackers = []
    for _ in range(predictor.dataset.bs):
        tracker = ns["create_tracker"](predictor.custom_args.tracking_method, cfg,
                                       predictor.custom_args.reid_model, predictor.device,
                                       predictor.custom_args.half,
                                       predictor.custom_args.per_class)
        if hasattr(tracker, "model"):
            tracker.model.warmup()
        trackers.append(tracker)
    predictor.trackers = trackers


def predictor(method, reid_model, bs=2, device="cuda:0", half=False, per_class=False):
    return SimpleNamespace(
        custom_args=SimpleNamespace(tracking_method=method, reid_model=reid_model, half=half,
                                    per_class=per_class),
        dataset=SimpleNamespace(bs=bs), device=device)
