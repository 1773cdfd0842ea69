"""ReID crop preprocessing + feature normalisation on the device (reference:
boxmot/appearance/reid_multibackend.py)."""
from .reid_multibackend import ReIDDetectMultiBackend, crop_rects, preprocess_host  # noqa: F401


def build_reid(reid, weights, device, half):
    """The trackers' ReID producer: `reid` when given, else ReIDDetectMultiBackend(weights,
    device, half) as the reference's trackers build it (bot_sort.py:217-219,
    deep_ocsort.py:343-345, hybridsort.py:344-346) when `weights` names a file (str / Path),
    else None (the caller passes embeddings to update).  A weights path that does not exist
    raises FileNotFoundError (the reference downloads it or exits, reid_multibackend.py:61-72)."""
    import os
    if reid is not None:
        return reid
    if weights is None or not isinstance(weights, (str, os.PathLike)):
        return None
    return ReIDDetectMultiBackend(weights, device, half)
