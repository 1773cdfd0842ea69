"""CMC estimators feeding BoT-SORT / DeepOCSORT's camera-motion warp.

Reference: BoTSORT always builds SparseOptFlow() (boxmot/trackers/botsort/bot_sort.py:228) and
DeepOCSort builds get_cmc_method('sof')() (deep_ocsort.py:351); both call cmc.apply(img, dets)
once per frame (bot_sort.py:293, deep_ocsort.py:391) and apply the returned 2x3 affine to every
track (multi_gmc / apply_affine_correction), which the device engines do.
"""
import warnings

import numpy as np


class IdentityCMC:
    """Static-camera motion model: the identity warp every frame."""

    def apply(self, img, dets):
        return np.eye(2, 3)


_warned = set()


def default_cmc(owner):
    """The estimator a tracker gets when the caller passes no `cmc=`.

    The reference estimates the warp with OpenCV's sparse optical flow; this build has no such
    estimator on the default path, so the identity warp is used and a one-time warning says so:
    on a moving camera the tracks then differ from the reference's.  Pass `cmc=IdentityCMC()`
    to state a static camera explicitly (no warning), or any object with apply(img, dets) -> 2x3.
    """
    if owner not in _warned:
        _warned.add(owner)
        warnings.warn(
            f"{owner}: no cmc= estimator given; the reference runs SparseOptFlow here "
            "(bot_sort.py:228, deep_ocsort.py:351). Using the identity warp (static camera): on a "
            "moving camera the tracks differ from the reference's. Pass cmc=IdentityCMC() to "
            "silence this, or an object with apply(img, dets) -> 2x3 warp.",
            RuntimeWarning, stacklevel=3)
    return IdentityCMC()
