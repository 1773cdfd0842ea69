"""Paths mirroring boxmot/utils/__init__.py:8-13 (ROOT, BOXMOT, EXAMPLES, WEIGHTS, REQUIREMENTS).

ROOT is the repository root; the tracker YAMLs live at ROOT/'boxmot'/'configs' (the `boxmot`
alias package), where the reference keeps them and where examples/track.py:37-41 looks.
"""
from pathlib import Path

FILE = Path(__file__).resolve()
ROOT = FILE.parents[2]                 # repository root
BOXMOT = ROOT / "boxmot"               # the alias package; holds configs/
EXAMPLES = ROOT / "examples"
WEIGHTS = ROOT / "examples" / "weights"
REQUIREMENTS = ROOT / "requirements.txt"
