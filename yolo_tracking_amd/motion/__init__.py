"""Camera-motion compensation producers (reference: boxmot/motion/cmc/)."""
from .cmc import IdentityCMC, default_cmc

__all__ = ["IdentityCMC", "default_cmc"]
