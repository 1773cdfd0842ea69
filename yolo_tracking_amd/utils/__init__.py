"""Paths mirroring boxmot/utils/__init__.py:8-13 (ROOT, BOXMOT, WEIGHTS ...)."""
from pathlib import Path

FILE = Path(__file__).resolve()
ROOT = FILE.parents[2]                 # repository root
BOXMOT = ROOT / "yolo_tracking_amd"    # package directory (holds configs/)
EXAMPLES = ROOT / "examples"
WEIGHTS = ROOT / "examples" / "weights"
