"""Correlation blocks: dense all-pairs pyramid and the memory-efficient local path.

``CorrPyramid`` is the MI355X replacement for the reference ``CorrBlock``
(core/corr.py:12-50) and ``LocalCorrPyramid`` for ``AlternateCorrBlock``
(core/corr.py:63-91).  Both expose ``__call__(coords) -> (B, L*(2r+1)^2, H, W)``.

Autograd design of the dense path (GPU):

* ``_BuildPyramid`` runs the bf16 MFMA GEMM (``raft_amd::gemm_nt``, fp32
  accumulate, 1/sqrt(C) in the epilogue) and the pyramid pools once per
  forward.  Its only differentiable output is a scalar *token*.
* every refinement iteration calls ``_Lookup(token, coords)``.  Its backward
  does not return a dense pyramid gradient: it accumulates, in place and
  without atomics, into one shared fp32 pyramid-gradient buffer owned by the
  pyramid state, and returns a zero token gradient.
* autograd runs ``_BuildPyramid.backward`` only after every lookup's backward
  has run (they all feed the token), so it folds the accumulated 4-level
  gradient to level 0 once, and runs two MFMA GEMMs for dfmap1/dfmap2.

The reference instead materialises a full-pyramid ``grid_sample`` gradient
per iteration and sums them (12 dense buffers per training step).
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn.functional as F

from . import reference as ref
from ._ext import ops, use_native


def _pad_to(n: int, m: int) -> int:
    return (n + m - 1) // m * m


class _PyramidState:
    """Forward/backward state shared by a pyramid build and its lookups."""

    def __init__(self, num_levels: int, radius: int):
        self.num_levels = num_levels
        self.radius = radius
        self.levels: List[torch.Tensor] = []
        self.dlevels: Optional[List[torch.Tensor]] = None
        self.shape = None

    def grad_buffers(self) -> List[torch.Tensor]:
        if self.dlevels is None:
            self.dlevels = [torch.zeros_like(l) for l in self.levels]
        return self.dlevels

    def release(self):
        self.levels = []
        self.dlevels = None


class _BuildPyramid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fmap1, fmap2, state: _PyramidState):
        B, C, H, W = fmap1.shape
        HW = H * W
        k = ops()
        f1 = fmap1.detach().permute(0, 2, 3, 1).to(torch.bfloat16).reshape(B, HW, C).contiguous()
        f2 = fmap2.detach().permute(0, 2, 3, 1).to(torch.bfloat16).reshape(B, HW, C).contiguous()
        if C % 64 != 0:
            pad = _pad_to(C, 64) - C
            f1 = F.pad(f1, (0, pad))
            f2 = F.pad(f2, (0, pad))
        corr = k.gemm_nt(f1, f2, 1.0 / math.sqrt(C), torch.float32)
        lvl = corr.view(B * HW, H, W)
        levels = [lvl]
        for _ in range(state.num_levels - 1):
            lvl = k.avgpool2x2(lvl)
            levels.append(lvl)
        state.levels = levels
        state.shape = (B, C, H, W)
        ctx.state = state
        ctx.save_for_backward(fmap1, fmap2)
        return fmap1.new_zeros((), dtype=torch.float32)

    @staticmethod
    def backward(ctx, gtoken):
        state: _PyramidState = ctx.state
        fmap1, fmap2 = ctx.saved_tensors
        if state.dlevels is None:
            state.release()
            return None, None, None
        B, C, H, W = state.shape
        HW = H * W
        ldp = _pad_to(HW, 64)
        k = ops()
        dC, dCt = k.pyramid_grad_combine(state.dlevels, B, H, W, ldp, 1.0 / math.sqrt(C))
        state.release()

        def nchw_pad(f):
            f = f.detach().reshape(B, C, HW).to(torch.bfloat16)
            return F.pad(f, (0, ldp - HW)).contiguous()

        g1 = k.gemm_nt(dC, nchw_pad(fmap2), 1.0, torch.float32)  # (B, HW, C)
        g2 = k.gemm_nt(dCt, nchw_pad(fmap1), 1.0, torch.float32)
        g1 = g1.view(B, H, W, C).permute(0, 3, 1, 2)
        g2 = g2.view(B, H, W, C).permute(0, 3, 1, 2)
        return g1.to(fmap1.dtype), g2.to(fmap2.dtype), None


class _Lookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, coords, state: _PyramidState, out_dtype, out_channels=0):
        coords = coords.detach().float().contiguous()
        out = ops().corr_lookup(state.levels, coords, state.radius, out_dtype, out_channels)
        ctx.state = state
        ctx.save_for_backward(coords)
        return out

    @staticmethod
    def backward(ctx, gout):
        (coords,) = ctx.saved_tensors
        state: _PyramidState = ctx.state
        if state.levels:
            ops().corr_lookup_backward_(state.grad_buffers(), coords, gout.contiguous(), state.radius)
        return torch.zeros((), device=gout.device), None, None, None, None


class CorrPyramid:
    """All-pairs correlation pyramid with radius-``radius`` lookup.

    GPU: native HIP/MFMA path (see module docstring).  CPU: reference ops.
    ``out_dtype`` selects the dtype of the looked-up features (bf16 under
    autocast feeds the motion encoder without an extra cast).
    """

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4):
        self.num_levels = num_levels
        self.radius = radius
        self.native = use_native(fmap1)
        if self.native:
            self.state = _PyramidState(num_levels, radius)
            self.token = _BuildPyramid.apply(fmap1, fmap2, self.state)
        else:
            corr = ref.corr_volume(fmap1.float(), fmap2.float())
            self.pyramid = ref.build_pyramid(corr, num_levels)

    def lookup_padded(self, coords: torch.Tensor, out_channels: int, out_dtype=torch.bfloat16) -> torch.Tensor:
        """Native only: (B, H, W, out_channels) NHWC features, zero beyond L*(2r+1)^2
        (the K padding the fused motion encoder's 1x1 conv expects)."""
        return _Lookup.apply(self.token, coords, self.state, out_dtype, out_channels)

    def __call__(self, coords: torch.Tensor, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        if self.native:
            dt = out_dtype or torch.float32
            out = _Lookup.apply(self.token, coords, self.state, dt, 0)
            return out.permute(0, 3, 1, 2)  # channels-last view (B, Ch, H, W)
        out = ref.pyramid_lookup(self.pyramid, coords, self.radius)
        return out if out_dtype is None else out.to(out_dtype)


# --------------------------------------------------------------------- local path
class _LocalCorr(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f1, f2, coords, radius: int, scale: float):
        coords = coords.detach().float().contiguous()
        out = ops().local_corr(f1, f2, coords, radius, scale)
        ctx.save_for_backward(f1, f2, coords)
        ctx.radius, ctx.scale = radius, scale
        return out

    @staticmethod
    def backward(ctx, gout):
        f1, f2, coords = ctx.saved_tensors
        g1, g2 = ops().local_corr_backward(f1, f2, coords, gout, ctx.radius, ctx.scale)
        return g1.to(f1.dtype), g2.to(f2.dtype), None, None, None


class LocalCorrPyramid:
    """Memory-efficient correlation: no HW x HW volume is ever stored.

    Pools fmap2 (not the volume; equivalent by linearity) into ``num_levels``
    levels once, and per lookup computes the (2r+1)^2 window correlations on
    the fly with the HIP ``local_corr`` kernel (fwd + bwd, so unlike the
    reference's alt_cuda_corr path this one can train).
    """

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 feature_dtype: Optional[torch.dtype] = None):
        self.num_levels = num_levels
        self.radius = radius
        self.native = use_native(fmap1)
        self.C = fmap1.shape[1]
        if self.native:
            dt = feature_dtype or torch.float32
            self.f1 = fmap1.permute(0, 2, 3, 1).to(dt).contiguous()
            f2 = fmap2
            self.f2 = []
            for i in range(num_levels):
                if i > 0:
                    f2 = F.avg_pool2d(f2, 2, stride=2)
                self.f2.append(f2.permute(0, 2, 3, 1).to(dt).contiguous())
        else:
            self.fmap1 = fmap1.float()
            self.fmap2 = [fmap2.float()]
            for i in range(1, num_levels):
                self.fmap2.append(F.avg_pool2d(self.fmap2[-1], 2, stride=2))

    def __call__(self, coords: torch.Tensor, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        scale = 1.0 / math.sqrt(self.C)
        outs = []
        for i in range(self.num_levels):
            ci = coords / (2 ** i)
            if self.native:
                o = _LocalCorr.apply(self.f1, self.f2[i], ci.detach().contiguous(), self.radius, scale)
                outs.append(o)  # (B, H, W, win)
            else:
                outs.append(ref.local_corr(self.fmap1, self.fmap2[i], ci, self.radius).permute(0, 2, 3, 1) * scale)
        out = torch.cat(outs, dim=-1).permute(0, 3, 1, 2)
        return out if out_dtype is None else out.to(out_dtype)
