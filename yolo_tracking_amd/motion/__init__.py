"""Camera-motion compensation producers (reference: boxmot/motion/cmc/)."""
from .cmc import IdentityCMC, default_cmc, get_cmc_method
from .ecc import ECC, EccEngine
from .sof import SofEngine, SparseOptFlow

__all__ = ["ECC", "EccEngine", "IdentityCMC", "SofEngine", "SparseOptFlow", "default_cmc",
           "get_cmc_method"]
