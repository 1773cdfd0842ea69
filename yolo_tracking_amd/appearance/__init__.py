"""ReID crop preprocessing + feature normalisation on the device (reference:
boxmot/appearance/reid_multibackend.py)."""
from .reid_multibackend import ReIDDetectMultiBackend, crop_rects, preprocess_host  # noqa: F401
