"""Query-pixel sharding of the all-pairs correlation (the context-parallel analogue for
high-resolution inference; SURVEY.md section 5, "Long-context / sequence parallelism").

RAFT's "sequence length" is the pixel count N = (H/8)(W/8): the correlation volume and its
pyramid are O(N^2) (reference core/corr.py:12-60 builds all of it on one device; its only
other option is the O(N) local correlation, core/corr.py:63-91).  Every row of the volume
belongs to ONE query pixel and the lookup of a query reads only its own row, so the volume
shards over query pixels with no halo exchange at all:

* each rank of the group keeps fmap2 whole (both feature maps are computed replicated, or
  all-gathered by the caller) and builds the pyramid rows of its contiguous range of query
  pixels only -- volume memory per GPU drops by the group size;
* per refinement iteration each rank samples the windows of its own queries and the
  (B, L*(2r+1)^2, n) features are all-gathered over the group (RCCL over xGMI on GPUs:
  B * N * 324 * 4 bytes per iteration, e.g. 42 MB at 1080p), after which every rank runs
  the (cheap, replicated) update block on the full image.

On the GPU both halves run on the native kernels of the dense path (ops/corr.py): the
rank's rows are ONE MFMA GEMM of its query rows of fmap1 against the pooled-fmap2 operand
(csrc/corr_volume.hip; bf16 volume under AMP, split-bf16 fp32-faithful otherwise), stored in
the blocked level layout, and the lookup is the dense lookup kernel over those rows (the
shard is presented to it as a 1 x n image of queries).  The features are all-gathered in the
dtype the update block consumes (bf16 under AMP: half the xGMI bytes).  On the CPU (tests)
the reference op sequence stands in.

Inference only (the all-gather carries no gradient).  Lookup semantics are those of the
reference CorrBlock (ops/reference.py pyramid_lookup), so the sharded model's output equals
the unsharded one up to float summation order (tests/test_query_shard_cpu.py,
tests/test_model_gpu.py).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import reference as ref
from ..ops._ext import ops, use_native


def shard_range(n: int, rank: int, world: int) -> tuple:
    """Contiguous, balanced [lo, hi) of ``n`` items for ``rank`` (sizes differ by <= 1)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


class ShardedCorrPyramid:
    """Drop-in for the model's ``corr_fn``: ``__call__(coords, out_dtype=None)`` returns the
    (B, L*(2r+1)^2, H, W) lookup features of ALL query pixels; this rank stores only the
    pyramid rows of its own queries."""

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 group: Optional[dist.ProcessGroup] = None, split: bool = True):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.radius = radius
        B, C, H, W = fmap1.shape
        self.shape = (B, H, W)
        self.lo, self.hi = shard_range(H * W, self.rank, self.world)
        self.counts = [shard_range(H * W, r, self.world) for r in range(self.world)]
        n = self.hi - self.lo
        self.native = use_native(fmap1)
        if self.native:
            self._build_native(fmap1, fmap2, num_levels, bool(split))
            return
        f1 = fmap1.float().reshape(B, C, H * W)[:, :, self.lo:self.hi].transpose(1, 2)  # (B, n, C)
        f2 = fmap2.float().reshape(B, C, H * W)
        corr = torch.matmul(f1, f2) / (C ** 0.5)  # (B, n, H*W): this rank's rows of the volume
        self.pyramid = ref.build_pyramid(corr.reshape(B * n, 1, H, W), num_levels)

    def _build_native(self, fmap1, fmap2, num_levels: int, split: bool):
        """This rank's rows of every level: one MFMA GEMM (ops/corr.py _BuildPyramid's layout)."""
        from ..ops.corr import _PyramidState

        B, C, H, W = fmap1.shape
        n = self.hi - self.lo
        st = _PyramidState(num_levels, self.radius)
        off = 0
        for l in range(num_levels):
            Hl, Wl = H >> l, W >> l
            st.sizes.append((Hl, Wl, off))
            off += -(-Wl // 16) * 16 * Hl
        st.ld = ld = off
        dt = torch.float32 if split else torch.bfloat16
        k = ops()
        f1 = fmap1.detach().permute(0, 2, 3, 1).reshape(B, H * W, C)[:, self.lo:self.hi].to(dt).contiguous()
        f2cat = k.pyramid_operand(fmap2.detach(), st.segments(), ld, True, False).to(dt)
        buf = torch.empty(B * n, ld, device=fmap1.device, dtype=dt)
        if n > 0:
            k.corr_gemm(f1, f2cat, buf, n, ld, C, B, C, n * C, C, ld * C, ld, n * ld, 1.0 / C ** 0.5, False, split, 0)
        st.buf = buf
        st.levels = st.views(buf)
        self.state = st
        self.feat_dtype = dt

    def local_lookup(self, coords: torch.Tensor) -> torch.Tensor:
        """(B, F, n) features of this rank's queries."""
        B, H, W = self.shape
        c = coords.float().reshape(B, 2, H * W)[:, :, self.lo:self.hi].unsqueeze(2)  # (B, 2, 1, n)
        if self.native:  # the shard's queries as a (B, 1, n) image of the dense lookup kernel
            st = self.state
            out = ops().corr_lookup(st.levels, c.contiguous(), self.radius, self.feat_dtype, 0)  # (B, 1, n, F)
            return out.reshape(B, self.hi - self.lo, -1).transpose(1, 2)
        return ref.pyramid_lookup(self.pyramid, c, self.radius).reshape(B, -1, self.hi - self.lo)

    def __call__(self, coords: torch.Tensor, out_dtype=None) -> torch.Tensor:
        B, H, W = self.shape
        local = self.local_lookup(coords)
        if out_dtype is not None and self.native:
            local = local.to(out_dtype)  # gather in the consumer's dtype (bf16 under AMP)
        if self.world > 1:
            nmax = max(hi - lo for lo, hi in self.counts)
            buf = local.new_zeros(B, local.shape[1], nmax)
            buf[:, :, :local.shape[2]] = local
            parts: List[torch.Tensor] = [torch.empty_like(buf) for _ in range(self.world)]
            dist.all_gather(parts, buf.contiguous(), group=self.group)
            local = torch.cat([p[:, :, :hi - lo] for p, (lo, hi) in zip(parts, self.counts)], dim=2)
        out = local.reshape(B, -1, H, W)
        return out.to(out_dtype) if out_dtype is not None else out

    def volume_bytes(self) -> int:
        """Bytes of this rank's pyramid (the O(N^2 / world) part)."""
        if self.native:
            return self.state.buf.numel() * self.state.buf.element_size()
        return sum(t.numel() * t.element_size() for t in self.pyramid)
