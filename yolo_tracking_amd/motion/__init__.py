"""Camera-motion compensation producers (reference: boxmot/motion/cmc/)."""
from .cmc import IdentityCMC, default_cmc, get_cmc_method
from .sof import SofEngine, SparseOptFlow

__all__ = ["IdentityCMC", "SofEngine", "SparseOptFlow", "default_cmc", "get_cmc_method"]
