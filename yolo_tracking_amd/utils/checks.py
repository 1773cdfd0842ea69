"""TestRequirements (boxmot/utils/checks.py:10-35): report missing packages, never install.

The reference's check_packages shells `pip install` for every requirement it cannot resolve and
calls exit() when that fails (:29-34); examples/track.py:15-16 calls it at import time for the
ultralytics fork.  There is no package index on an MI355X node of this build, so this version
reports (logger warning + `missing` list) and returns; nothing is downloaded or installed.
"""
import logging
from importlib import metadata

from . import REQUIREMENTS

logger = logging.getLogger("boxmot")


def _parse(req):
    from packaging.requirements import InvalidRequirement, Requirement
    try:
        return Requirement(str(req))
    except InvalidRequirement:
        return None


class TestRequirements:
    __test__ = False   # not a pytest test class

    def __init__(self):
        self.missing = []

    def check_requirements(self):
        """:12-14 — every line of REQUIREMENTS (comments skipped)."""
        lines = []
        if REQUIREMENTS.is_file():
            for ln in REQUIREMENTS.read_text().splitlines():
                ln = ln.split("#", 1)[0].strip()
                if ln:
                    lines.append(ln)
        return self.check_packages(lines)

    def check_packages(self, requirements, cmds=""):
        """:16-35 — each requirement must be installed at a matching version; the missing ones
        are logged and returned (and kept in self.missing), never pip-installed."""
        missing = []
        for r in requirements:
            req = _parse(r)
            if req is None:
                missing.append(str(r))
                continue
            try:
                version = metadata.version(req.name)
            except metadata.PackageNotFoundError:
                missing.append(str(r))
                continue
            if req.specifier and not req.specifier.contains(version, prereleases=True):
                missing.append(str(r))
        if missing:
            logger.warning("Missing packages: %s (no package index on this node: not installing%s)",
                           " ".join(f'"{m}"' for m in missing), f"; {cmds}" if cmds else "")
        self.missing = missing
        return missing
