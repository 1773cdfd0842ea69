"""CMC estimators feeding BoT-SORT / DeepOCSORT's camera-motion warp.

Reference: BoTSORT always builds SparseOptFlow() (boxmot/trackers/botsort/bot_sort.py:228) and
DeepOCSort builds get_cmc_method('sof')() (deep_ocsort.py:351); both call cmc.apply(img, dets)
once per frame (bot_sort.py:293, deep_ocsort.py:391) and apply the returned 2x3 affine to every
track (multi_gmc / apply_affine_correction), which the device engines do.  The default estimator
here is the same SparseOptFlow, on the GPU (motion/sof.py, csrc/cmc.hip).
"""
import numpy as np

from .ecc import ECC
from .sof import SparseOptFlow


class IdentityCMC:
    """Static-camera motion model: the identity warp every frame (pass cmc=IdentityCMC() to
    skip camera-motion estimation)."""

    def apply(self, img, dets):
        return np.eye(2, 3)


def get_cmc_method(cmc_method):
    """boxmot.motion.cmc.get_cmc_method (motion/cmc/__init__.py:9-19): the estimator class by
    name.  SparseOptFlow (what BoTSORT and DeepOCSort build) and ECC (what HybridSORT builds) run on
    the device; ORB / SIFT (OpenCV feature matchers no in-scope tracker uses) are refused."""
    if cmc_method in ("sof", "sparseOptFlow"):
        return SparseOptFlow
    if cmc_method == "ecc":
        return ECC
    raise NotImplementedError(f"cmc method {cmc_method!r}: 'sof' (SparseOptFlow) and 'ecc' (ECC) "
                              "are on the MI355X path")


def default_cmc(owner=None, device=0):
    """The estimator a tracker gets when the caller passes no `cmc=`: SparseOptFlow(), as in the
    reference (bot_sort.py:228, deep_ocsort.py:351)."""
    return SparseOptFlow(device=device)
