"""Whole training step replayed as HIP graph(s).

One RAFT training step at FlyingChairs size is ~1900 kernels (encoders, the
correlation pyramid, 12 x {lookup, 12 fused update convs, upsample}, the same
again backwards, loss, clip, AdamW).  Many of them are tiny, so host launch
cost and inter-kernel bubbles are a visible share of the step.  This module
captures

    zero grads -> forward -> sequence loss -> backward -> clip -> AdamW

into one HIP graph and replays it; with more than one rank the graph is split
around a single flat-buffer gradient all-reduce over RCCL (xGMI):

    graph A: zero grads, forward, loss, backward        (grads land in one flat fp32 buffer)
    eager  : all_reduce(flat grads)                       (one 21 MB collective, per-link bound)
    graph B: 1/world scale, clip, fused AdamW

The reference runs the same step eagerly through ``nn.DataParallel``
(train.py:161-183); semantics are identical (clip-norm, AdamW, OneCycle -- the
scheduler writes the on-device lr tensor between replays).

Requirements: static shapes (fixed crop/batch), an optimizer built with
``capturable=True`` and a tensor lr (``train.optim.fetch_optimizer(...,
capturable=True)``), no GradScaler (bf16).  Inputs are copied into static
buffers before each replay; outputs (loss, metrics) are views of graph memory
that the next replay overwrites.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

# one process: the gradients are the tensors the captured backward allocates (autograd steals
# them: no accumulate kernels; a pre-bound flat buffer costs one add kernel per parameter and
# measured no faster, profiles/r5n_bench_graph_flat.json).  The graphs are captured and replayed
# at default priority: on the high-priority step stream the replay ran 284-292 vs 402 pairs/s
# (profiles/r5n_bench_graph*.json).


class GraphedTrainStep:
    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer,
                 loss_fn: Callable, iters: int, clip: float = 1.0, gamma: float = 0.8,
                 process_group=None, warmup: int = 3, enabled: bool = True):
        self.model = model
        if enabled:
            model.autocast_cache = False  # see RAFT._autocast
        self.optimizer = optimizer
        self.loss_fn = loss_fn
        self.iters = iters
        self.clip = clip
        self.gamma = gamma
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self.warmup = warmup
        self.enabled = enabled
        self.params: List[torch.nn.Parameter] = [p for p in model.parameters() if p.requires_grad]
        self.flat: Optional[torch.Tensor] = None
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.static_in: Optional[List[torch.Tensor]] = None
        self.out: Optional[Tuple[torch.Tensor, Dict[str, torch.Tensor], torch.Tensor]] = None
        self.skipped: Optional[torch.Tensor] = None
        if self.world > 1:  # no DDP wrapper here: start every rank from rank 0's weights
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, 0, group=process_group)

    # -------------------------------------------------------------- step pieces
    def _bind_flat_grads(self):
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        o = 0
        for p in self.params:
            n = p.numel()
            # same strides as the parameter (channels-last convs): fused AdamW wants matching layouts
            assert p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))
            p.grad = self.flat.as_strided(p.shape, p.stride(), o)
            o += n

    def _use_flat(self) -> bool:
        return self.world > 1 or not self.params[0].is_cuda

    def _grads(self) -> List[torch.Tensor]:
        return [p.grad for p in self.params if p.grad is not None]

    def _fwd_bwd(self, image1, image2, flow, valid):
        if self.flat is not None:
            self.flat.zero_()
        else:
            for p in self.params:  # the backward allocates (in the graph's pool when captured)
                p.grad = None
        preds = self.model(image1, image2, iters=self.iters)
        loss, metrics = self.loss_fn(preds, flow, valid, self.gamma)
        loss.backward()
        return loss, metrics

    def _update(self):
        if self.world > 1:
            self.flat.div_(self.world)
        if self.flat is not None:
            norm = torch.linalg.vector_norm(self.flat)
            coef = (self.clip / (norm + 1e-6)).clamp(max=1.0)
            self.flat.mul_(coef)
        else:
            grads = self._grads()
            norm = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(grads)))
            coef = (self.clip / (norm + 1e-6)).clamp(max=1.0)
            torch._foreach_mul_(grads, coef)
        # failure guard without a host sync: a non-finite norm makes fused AdamW a no-op
        bad = (~torch.isfinite(norm)).float()
        self.skipped.add_(bad)
        if self.optimizer.defaults.get("fused"):
            self.optimizer.found_inf = bad
            self.optimizer.step()
            self.optimizer.found_inf = None
        elif not bool(bad):  # CPU / non-fused: host check (never captured)
            self.optimizer.step()
        return norm

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat, group=self.pg)

    def _eager(self, image1, image2, flow, valid):
        loss, metrics = self._fwd_bwd(image1, image2, flow, valid)
        self._allreduce()
        norm = self._update()
        return loss, metrics, norm

    # -------------------------------------------------------------- capture
    def _snapshot(self):
        """Model parameters/buffers and optimizer state before the warm-up steps."""
        model_state = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        opt_state = {id(p): {k: v.detach().clone() if torch.is_tensor(v) else v
                             for k, v in self.optimizer.state[p].items()}
                     for p in self.params if p in self.optimizer.state}
        return model_state, opt_state

    @torch.no_grad()
    def _restore(self, snap):
        """Undo the warm-up steps in place (graph addresses stay valid)."""
        model_state, opt_state = snap
        for k, v in self.model.state_dict().items():
            v.copy_(model_state[k])
        for p in self.params:
            st = self.optimizer.state.get(p)
            if not st:
                continue
            old = opt_state.get(id(p))
            for k, v in st.items():
                if torch.is_tensor(v):
                    v.copy_(old[k]) if old is not None else v.zero_()

    def _capture(self, batch):
        dev = self.params[0].device
        self.static_in = [t.detach().clone() for t in batch]
        if self._use_flat():
            self._bind_flat_grads()
        self.skipped = torch.zeros((), device=dev)
        snap = self._snapshot()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(self.warmup):  # lazy init, MIOpen find, allocator warm-up
                self._eager(*self.static_in)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self._restore(snap)
        self.skipped.zero_()
        pool = torch.cuda.graph_pool_handle()
        ga = torch.cuda.CUDAGraph()
        # capture on the warm-up stream: autograd's AccumulateGrad nodes remember the stream
        # they were created on, and a mismatch would move gradient accumulation off the capture
        with torch.cuda.graph(ga, pool=pool, stream=side):
            loss, metrics = self._fwd_bwd(*self.static_in)
            if self.world == 1:
                norm = self._update()
        self.graphs = [ga]
        if self.world > 1:
            gb = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gb, pool=pool, stream=side):
                norm = self._update()
            self.graphs.append(gb)
        self.out = (loss.detach(), metrics, norm)

    def __call__(self, image1, image2, flow, valid):
        """One optimizer step; returns (loss, metrics, grad_norm) device tensors."""
        batch = (image1, image2, flow, valid)
        if not (self.enabled and image1.is_cuda):
            if self.skipped is None:
                if self._use_flat():
                    self._bind_flat_grads()
                self.skipped = torch.zeros((), device=image1.device)
            return self._eager(*batch)
        if self.static_in is None:
            self._capture(batch)
        else:
            for s, t in zip(self.static_in, batch):
                if s.data_ptr() != t.data_ptr():
                    s.copy_(t, non_blocking=True)
        self._replay()
        return self.out

    def _replay(self):
        self.graphs[0].replay()
        if self.world > 1:
            self._allreduce()
            self.graphs[1].replay()
