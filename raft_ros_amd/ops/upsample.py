"""Flow upsampling ops: fused convex 8x upsampling (HIP) and bilinear ``upflow8``.

Reference: RAFT.upsample_flow (core/raft.py:72-83) and upflow8
(core/utils/utils.py:80-82).
"""
from __future__ import annotations

import torch

from . import reference as ref
from ._ext import ops, use_native


class _ConvexUpsample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flow, mask):
        flow = flow.float().contiguous()
        out = ops().convex_upsample(flow, mask)
        ctx.save_for_backward(flow, mask)
        return out

    @staticmethod
    def backward(ctx, gout):
        flow, mask = ctx.saved_tensors
        dflow, dmask = ops().convex_upsample_backward(flow, mask, gout)
        return dflow, dmask


def convex_upsample(flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """(B, 2, H, W) flow + (B, 576, H, W) mask logits -> (B, 2, 8H, 8W) fp32 flow."""
    if use_native(flow):
        return _ConvexUpsample.apply(flow, mask)
    return ref.convex_upsample(flow.float(), mask.float())


class _Upflow8(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flow):
        ctx.hw = flow.shape[-2:]
        return ops().upflow8(flow.float().contiguous())

    @staticmethod
    def backward(ctx, gout):
        H, W = ctx.hw
        return ops().upflow8_backward(gout.float().contiguous(), H, W, None)


def upflow8(flow: torch.Tensor, mode: str = "bilinear") -> torch.Tensor:
    """8x bilinear (align_corners) upsampling of a (B, 2, H, W) flow, times 8 (HIP on GPU)."""
    if mode == "bilinear" and use_native(flow):
        return _Upflow8.apply(flow)
    return ref.upflow8(flow, mode)
