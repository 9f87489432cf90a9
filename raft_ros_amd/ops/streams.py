"""Auxiliary HIP streams shared by the concurrent branches of a RAFT step.

A process gets GPU_MAX_HW_QUEUES hardware queues (4 by default on MI355X); streams beyond
that share a queue and serialise behind each other.  A step therefore uses at most three
compute streams, leaving a queue for the RCCL communicator under DDP:

* the current (main) stream: the critical path;
* ``side``: the context encoder beside the feature encoder (forward and backward), and in
  the refinement loop's backward each step's upsampler / head data gradients (the context
  encoder is idle then);
* ``tail``: the refinement loop's work nobody waits for until the end -- the mask head and
  the upsampling in the forward, the motion-encoder and lookup backward;
* ``wgrad``: the batched update-block weight gradients of the iterations whose backward is
  complete, beside the remaining iterations' backward (ops/update_fused.py ``WGRAD_SPLIT``).
  Under DDP this fourth compute stream shares a hardware queue with the communicator's
  stream; the gradients it computes are what that communicator waits for anyway.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

_STREAMS: Dict[Tuple[torch.device, str], torch.cuda.Stream] = {}


def aux_stream(device, name: str) -> torch.cuda.Stream:
    """The process-wide ``name`` ('side' or 'tail') stream of ``device``."""
    if name not in ("side", "tail", "wgrad"):
        raise ValueError(f"unknown auxiliary stream {name!r}")
    key = (torch.device(device), name)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(device=key[0])
    return _STREAMS[key]
