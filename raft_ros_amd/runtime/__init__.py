"""Execution runtime helpers: HIP-graph replay of inference and of the whole training step."""
from .graphs import GraphedRAFT
from .train_graph import GraphedTrainStep

__all__ = ["GraphedRAFT", "GraphedTrainStep"]
