"""HIP-graph replay of RAFT inference.

A RAFT forward at inference resolution is a long chain of small kernels
(encoders, then ``iters`` x {lookup, ~12 update-block convs, upsample}); at
ROS / demo sizes the host launch cost is comparable to the GPU work.  Capturing
the whole forward once per input shape and replaying it removes that cost --
the HIP counterpart of the reference's plain eager loop
(ros/scripts/main.py:117-149, demo.py:42-63, evaluate.py:74-166).

Usage::

    runner = GraphedRAFT(model, iters=20)
    flow_low, flow_up = runner(image1, image2)      # same as model(..., test_mode=True)

Outputs are views of the graph's static buffers: they are overwritten by the
next call with the same shape (``clone()`` them to keep them).  Every shape has
its own memory pool, so replaying one shape never clobbers the outputs another
shape returned earlier.  Weight updates
in place (``load_state_dict``, optimizer steps) are picked up by the replay;
call :meth:`reset` after replacing parameter tensors.  On CPU (or with
``enabled=False``) the runner simply calls the model.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional, Tuple

import torch


class _Entry:
    __slots__ = ("graph", "in1", "in2", "init", "out")


class GraphedRAFT:
    def __init__(self, model: torch.nn.Module, iters: int = 12, max_graphs: int = 4, enabled: bool = True,
                 warmup: int = 2):
        self.model = model
        self.iters = iters
        self.max_graphs = max_graphs
        self.enabled = enabled
        self.warmup = warmup
        self._graphs: "OrderedDict[tuple, _Entry]" = OrderedDict()

    def reset(self) -> None:
        self._graphs.clear()

    @property
    def num_graphs(self) -> int:
        return len(self._graphs)

    def _eager(self, image1, image2, flow_init):
        return self.model(image1, image2, iters=self.iters, flow_init=flow_init, test_mode=True)

    @torch.no_grad()
    def __call__(self, image1: torch.Tensor, image2: torch.Tensor,
                 flow_init: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        if not (self.enabled and image1.is_cuda):
            return self._eager(image1, image2, flow_init)
        key = (tuple(image1.shape), image1.dtype, image1.device, flow_init is not None,
               None if flow_init is None else tuple(flow_init.shape))
        e = self._graphs.get(key)
        if e is None:
            e = self._capture(image1, image2, flow_init)
            self._graphs[key] = e
            while len(self._graphs) > self.max_graphs:
                self._graphs.popitem(last=False)
        else:
            self._graphs.move_to_end(key)
            e.in1.copy_(image1)
            e.in2.copy_(image2)
            if flow_init is not None:
                e.init.copy_(flow_init)
        e.graph.replay()
        return e.out

    def _capture(self, image1, image2, flow_init) -> _Entry:
        e = _Entry()
        e.in1 = image1.clone()
        e.in2 = image2.clone()
        e.init = None if flow_init is None else flow_init.clone()
        side = torch.cuda.Stream(device=image1.device)
        side.wait_stream(torch.cuda.current_stream(image1.device))
        with torch.cuda.stream(side):
            for _ in range(self.warmup):  # allocator / lazy-init warm-up outside the capture
                self._eager(e.in1, e.in2, e.init)
        torch.cuda.current_stream(image1.device).wait_stream(side)
        # a private pool per shape: a later capture must not place its temporaries in
        # memory that holds the outputs of an earlier shape's graph
        e.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(e.graph, pool=torch.cuda.graph_pool_handle()):
            e.out = self._eager(e.in1, e.in2, e.init)
        return e
