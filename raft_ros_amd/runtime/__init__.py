"""Execution runtime helpers: HIP-graph inference replay."""
from .graphs import GraphedRAFT

__all__ = ["GraphedRAFT"]
