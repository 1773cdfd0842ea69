"""`boxmot`: the reference's import paths over the MI355X package (a drop-in alias).

The reference's package (boxmot/__init__.py:5-18) and the module paths its users and
`examples/track.py:9-12` import resolve here to the modules of `yolo_tracking_amd` — the same
module objects for every leaf module (a package path that also has alias children is a
forwarding node over the real package), so the classes, the process-global ID counters and the
loaded C-ABI library are shared — and the tracker YAMLs live at `ROOT/'boxmot'/'configs'` exactly where
`examples/track.py:37-41` builds their paths (ROOT = boxmot.utils.ROOT = the repository root).

    import boxmot                                  # registers every alias below
    from boxmot import TRACKERS
    from boxmot.tracker_zoo import create_tracker
    from boxmot.utils import ROOT, WEIGHTS
    from boxmot.utils.checks import TestRequirements

Importing boxmot imports every tracker module (and torch, through the ReID producer), as the
reference's package does.  Nothing here computes; there is no CPU fallback behind these names.
"""
import importlib
import sys
import types

import yolo_tracking_amd as _yta
from yolo_tracking_amd import (TRACKERS, BoTSORT, BYTETracker, DeepOCSort, HybridSORT,  # noqa: F401
                               OCSort, __version__, create_tracker, get_tracker_config, gsi)

OCSORT = OCSort          # boxmot/__init__.py:7 exports the OCSort class under this name
DeepOCSORT = DeepOCSort  # boxmot/__init__.py:8


class _StrongSORT:
    """boxmot/__init__.py:10: StrongSORT is outside the MI355X path."""

    def __init__(self, *a, **k):
        raise NotImplementedError("StrongSORT is not on the MI355X path; see DESIGN.md §7")


StrongSORT = _StrongSORT

# reference module path -> module of this build (boxmot/ tree of the reference, v10.0.51)
ALIASES = {
    "boxmot.tracker_zoo": "yolo_tracking_amd.tracker_zoo",
    "boxmot.utils": "yolo_tracking_amd.utils",
    "boxmot.utils.checks": "yolo_tracking_amd.utils.checks",
    "boxmot.trackers": "yolo_tracking_amd.trackers",
    "boxmot.trackers.bytetrack.byte_tracker": "yolo_tracking_amd.trackers.bytetrack",
    "boxmot.trackers.bytetrack.basetrack": "yolo_tracking_amd.trackers.basetrack",
    "boxmot.trackers.botsort.bot_sort": "yolo_tracking_amd.trackers.botsort",
    "boxmot.trackers.ocsort.ocsort": "yolo_tracking_amd.trackers.ocsort",
    "boxmot.trackers.deepocsort.deep_ocsort": "yolo_tracking_amd.trackers.deepocsort",
    "boxmot.trackers.hybridsort.hybridsort": "yolo_tracking_amd.trackers.hybridsort",
    "boxmot.postprocessing": "yolo_tracking_amd.postprocessing",
    "boxmot.postprocessing.gsi": "yolo_tracking_amd.postprocessing.gsi",
    "boxmot.appearance": "yolo_tracking_amd.appearance",
    "boxmot.appearance.reid_multibackend": "yolo_tracking_amd.appearance.reid_multibackend",
    "boxmot.motion": "yolo_tracking_amd.motion",
    "boxmot.motion.cmc": "yolo_tracking_amd.motion.cmc",
    "boxmot.motion.cmc.sof": "yolo_tracking_amd.motion.sof",
    "boxmot.motion.cmc.ecc": "yolo_tracking_amd.motion.ecc",
}


class _Forward(types.ModuleType):
    """A reference package path whose module of this build also has alias-only children (e.g.
    boxmot.trackers -> yolo_tracking_amd.trackers, with boxmot.trackers.bytetrack below it):
    attribute lookups fall through to the real module, while the alias children are attached
    here, never onto the real module (whose own submodule attributes stay untouched)."""

    def __init__(self, name, target):
        super().__init__(name, target.__doc__)
        self.__path__ = []
        self.__wrapped__ = target

    def __getattr__(self, attr):
        return getattr(self.__wrapped__, attr)


def _register():
    me = sys.modules[__name__]
    parents = {a.rsplit(".", 1)[0] for a in ALIASES}
    for alias in sorted(ALIASES, key=lambda a: a.count(".")):
        mod = importlib.import_module(ALIASES[alias])
        if any(p == alias or p.startswith(alias + ".") for p in parents):
            mod = _Forward(alias, mod)          # has alias children: a boxmot-owned node
        parts = alias.split(".")
        parent = me
        for depth in range(1, len(parts) - 1):   # reference-only intermediate packages
            name = ".".join(parts[:depth + 1])
            if name not in sys.modules:
                pkg = types.ModuleType(name, f"reference package path {name} (alias)")
                pkg.__path__ = []
                sys.modules[name] = pkg
                setattr(parent, parts[depth], pkg)
            parent = sys.modules[name]
        sys.modules[alias] = mod
        # only boxmot-owned modules (this package, alias namespaces, _Forward nodes) get
        # attributes: a yolo_tracking_amd module is never modified
        assert parent.__name__.startswith("boxmot"), parent.__name__
        setattr(parent, parts[-1], mod)


_register()

__all__ = ("__version__", "BYTETracker", "BoTSORT", "OCSORT", "DeepOCSORT", "HybridSORT",
           "StrongSORT", "create_tracker", "get_tracker_config", "gsi", "TRACKERS")
