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

import contextlib
import os
from typing import Dict, Tuple

import torch

_STREAMS: Dict[Tuple[torch.device, str], torch.cuda.Stream] = {}
_STEP: Dict[torch.device, torch.cuda.Stream] = {}


def step_stream(device) -> torch.cuda.Stream:
    """A high-priority stream for the training step itself (the main stream above).

    The refinement loop's critical chain (lookup -> motion encoder -> GRU -> heads, and its
    backward) runs on the main stream while the side / tail streams carry work it does not wait
    for; with the main stream at high priority the hardware scheduler dispatches its kernels
    ahead of queued side / tail kernels.  Measured +1.5 % at config #2 on MI355X (six
    interleaved A/B pairs, profiles/r4_bench_hp_ab.log)."""
    key = torch.device(device)
    if key not in _STEP:
        _STEP[key] = torch.cuda.Stream(device=key, priority=-1)
    return _STEP[key]


@contextlib.contextmanager
def step_context(device):
    """``with step_context(dev): <one training step>`` -- the step on :func:`step_stream`, ordered
    after the current stream's queued work, and the current stream ordered after the step on
    exit (so code outside -- validation, checkpoints, ``.item()`` -- sees its results).
    ``RAFT_HP_MAIN=0``: the current stream, no switch."""
    dev = torch.device(device)
    if dev.type != "cuda" or os.environ.get("RAFT_HP_MAIN", "1") == "0":
        yield
        return
    outer = torch.cuda.current_stream(dev)
    s = step_stream(dev)
    s.wait_stream(outer)
    try:
        with torch.cuda.stream(s):
            yield
    finally:
        outer.wait_stream(s)


def aux_stream(device, name: str) -> torch.cuda.Stream:
    """The process-wide ``name`` ('side' or 'tail') stream of ``device``."""
    if name not in ("side", "tail", "wgrad"):
        raise ValueError(f"unknown auxiliary stream {name!r}")
    key = (torch.device(device), name)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(device=key[0])
    return _STREAMS[key]


class LeadLimiter:
    """Bound how far the host runs ahead of the GPU: ``step_done()`` after issuing a step
    records an event on the current stream and waits for the one of ``max_lead`` steps ago.

    The eager training step issues its ~17 ms of host work per ~20 ms GPU step, so left alone
    the host drifts further ahead every step; the caching allocator then holds more and more
    blocks whose last use is still queued and keeps mapping new memory (10.9 -> 17.1 GiB
    reserved over 40 steps, host issue 12 -> 19 ms/step from allocator churn;
    profiles/r4_host_lead_unthrottled.log vs r4_host_lead_before_fix.log).  One or two steps of
    lead already keep the GPU fed (the step time is unchanged)."""

    def __init__(self, max_lead: int = 2):
        self.max_lead = max_lead
        self._events = []

    def step_done(self, device) -> None:
        dev = torch.device(device)
        if dev.type != "cuda" or self.max_lead <= 0:
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        self._events.append(ev)
        if len(self._events) > self.max_lead:
            self._events.pop(0).synchronize()
