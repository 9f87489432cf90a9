"""Fused ConvGRU gate math with autograd (HIP on GPU, PyTorch on CPU).

``gates_zr(zr, h) -> (z, r*h)`` and ``blend(z, q, h) -> (1-z) h + z tanh(q)``
replace the ~10 elementwise launches per GRU stage of the reference
(core/update.py:24-31, 43-58) with one kernel each way.
"""
from __future__ import annotations

import torch

from ._ext import get_backend, ops, use_native  # noqa: F401

_CL = torch.channels_last


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous(memory_format=_CL)


class _GatesZR(torch.autograd.Function):
    @staticmethod
    def forward(ctx, zr, h):
        zr, h = _cl(zr), _cl(h.to(zr.dtype))
        z, rh = ops().gru_gates(zr, h)
        ctx.save_for_backward(zr, h)
        ctx.h_dtype = h.dtype
        return z, rh

    @staticmethod
    def backward(ctx, gz, grh):
        zr, h = ctx.saved_tensors
        if gz is None:
            gz = torch.zeros_like(h)
        if grh is None:
            grh = torch.zeros_like(h)
        dzr, dh = ops().gru_gates_backward(zr, h, gz, grh)
        return dzr, dh


class _Blend(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, q, h):
        dt = q.dtype
        z, q, h = _cl(z.to(dt)), _cl(q), _cl(h.to(dt))
        out = ops().gru_blend(z, q, h)
        ctx.save_for_backward(z, q, h)
        return out

    @staticmethod
    def backward(ctx, g):
        z, q, h = ctx.saved_tensors
        dz, dq, dh = ops().gru_blend_backward(z, q, h, g)
        return dz, dq, dh


def gates_zr(zr: torch.Tensor, h: torch.Tensor):
    C = h.shape[1]
    if use_native(zr) and zr.dtype in (torch.bfloat16, torch.float32) and C % 8 == 0:
        return _GatesZR.apply(zr, h)
    z = torch.sigmoid(zr[:, :C])
    r = torch.sigmoid(zr[:, C:])
    return z, r * h


def blend(z: torch.Tensor, q: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    if use_native(q) and q.dtype in (torch.bfloat16, torch.float32) and q.numel() % 8 == 0:
        return _Blend.apply(z, q, h)
    return (1 - z) * h + z * torch.tanh(q)
