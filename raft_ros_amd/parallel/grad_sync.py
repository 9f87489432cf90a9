"""Data-parallel gradient averaging in a handful of launches (replaces DDP's reducer).

RAFT's gradients do not arrive the way DistributedDataParallel's bucketing assumes.  The
refinement loop's weight gradients are computed in ONE batched pass per layer after the last
step's backward (ops/update_fused.py ``WeightToken``), and the encoders' come right after -- so
nearly all 21 MB of fp32 gradients become ready within the last few milliseconds of the
backward, and there is little backward left for bucket all-reduces to hide behind.  What DDP
does cost is per parameter: its autograd hooks copy each of the ~200 gradients into a bucket
view (one copy kernel each), which measured +8 % step time at world size 1
(tests/test_ddp_gpu.py, RCCL, MI355X) before any byte crossed xGMI.

``GradSync`` instead lets autograd hand each parameter its freshly computed gradient (no
hook, no copy), then after ``backward()``:

  1. one ``_foreach_copy_`` (multi-tensor kernel, a few launches) packs every gradient into a
     persistent flat fp32 buffer -- the destinations are strided like the parameters
     (channels-last conv weights stay dense), so no layout conversion;
  2. one all-reduce of the flat buffer (RCCL ``AVG`` over xGMI; gloo: SUM + one scale);
  3. each ``p.grad`` becomes a view of its slice of the averaged buffer (no copy back).

A parameter that no rank computed a gradient for keeps ``p.grad = None`` (so AdamW skips
it, as in single-process training and DDP).  Which parameters receive gradients is found
on the first ``sync()``: a per-parameter "had a gradient" count rides in the same
all-reduce and is read back on the host that one time (RAFT uses every parameter in every
step; a rank with no sample of the global batch -- parallel/batching.py -- has no gradient
at all and sends zeros).  A later step in which a parameter marked unused has a local
gradient raises instead of silently dropping it; after a collective change of the trainable
set (unfreezing a branch) every rank calls ``reset_usage()`` and the next ``sync()`` finds
the flags again.

At 21 MB the ring all-reduce over 8 MI355X is ~0.1-0.2 ms: one large collective is the cheap
case on point-to-point xGMI links.  ``bf16=True`` halves the bytes on the wire (the buffer is
cast to bf16 for the all-reduce; each rank's contribution is rounded to bf16).

Parameters and buffers are broadcast from rank 0 once at construction (DDP's initial sync);
BatchNorm running statistics are not re-broadcast per step -- in training mode the batch
statistics are used and rank 0's checkpoint holds rank 0's running statistics either way (the
reference's DataParallel keeps the replica-0 ones too, train.py:138).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class GradSync:
    def __init__(self, model: torch.nn.Module, group=None, bf16: bool = False, broadcast: bool = True):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params: List[torch.nn.Parameter] = [p for p in model.parameters() if p.requires_grad]
        self.bf16 = bf16
        dev = self.params[0].device
        self.backend = dist.get_backend(group)
        total = sum(p.numel() for p in self.params)
        self.total = total
        # + one "had a gradient" slot per parameter (used by the first sync only)
        self.flat = torch.empty(total + len(self.params), device=dev, dtype=torch.float32)
        self.used: Optional[List[bool]] = None
        self.unused_idx: List[int] = []
        self.views: List[torch.Tensor] = []
        off = 0
        for p in self.params:
            if not _dense(p):
                raise ValueError("GradSync: parameters must be dense (contiguous or channels-last)")
            self.views.append(torch.as_strided(self.flat, p.shape, p.stride(), off))
            off += p.numel()
        self._zeros: Optional[List[torch.Tensor]] = None
        if broadcast and self.world > 1:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, 0, group=group)

    def reset_usage(self) -> None:
        """Re-detect on the next ``sync()`` which parameters receive gradients (collective:
        every rank calls it before the same step)."""
        self.used = None

    def sync(self) -> None:
        """Average ``p.grad`` over the ranks (call after ``backward()``, before unscale / clip /
        the optimizer).  A parameter without a gradient contributes zeros (every rank must
        send the same buffer) and gets the averaged gradient of the others; one that no rank
        has a gradient for stays ``None``."""
        first = self.used is None
        if not first:
            # host-only check (no sync): a gradient on a parameter found unused on the first
            # step would be dropped by the p.grad = None below
            for i in self.unused_idx:
                if self.params[i].grad is not None:
                    raise RuntimeError(
                        f"GradSync: parameter {i} received no gradient on any rank when usage was detected but has "
                        "one now; call reset_usage() on every rank after changing the set of trained parameters")
        if first:
            flags = torch.tensor([0.0 if p.grad is None else 1.0 for p in self.params], dtype=torch.float32)
            self.flat[self.total:].copy_(flags)
        n = self.flat.numel() if first else self.total
        grads = []
        for p, v in zip(self.params, self.views):
            g = p.grad
            if g is None:
                g = torch.zeros_like(v)
            elif g.dtype != torch.float32:
                g = g.float()
            grads.append(g)
        if all(g.stride() == v.stride() for g, v in zip(grads, self.views)):
            torch._foreach_copy_(self.views, grads)
        else:  # a gradient in another layout than its parameter: per-tensor strided copies
            for v, g in zip(self.views, grads):
                v.copy_(g)
        if self.world > 1:
            flat = self.flat[:n]
            if self.bf16:
                buf = flat.to(torch.bfloat16)
                dist.all_reduce(buf, group=self.group)
                flat.copy_(buf)
                flat.mul_(1.0 / self.world)
            elif self.backend == "nccl":
                dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=self.group)
            else:
                dist.all_reduce(flat, group=self.group)
                flat.mul_(1.0 / self.world)
        if first:  # one host read, on the first step only
            self.used = (self.flat[self.total:] > 0).tolist()
            self.unused_idx = [i for i, u in enumerate(self.used) if not u]
        for p, v, u in zip(self.params, self.views, self.used):
            p.grad = v if u else None


def _dense(p: torch.Tensor) -> bool:
    """Non-overlapping and dense: the strides are a permutation of a contiguous layout's."""
    dims = sorted((s, n) for s, n in zip(p.stride(), p.shape) if n != 1)
    expect = 1
    for s, n in dims:
        if s != expect:
            return False
        expect *= n
    return True
