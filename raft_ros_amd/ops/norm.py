"""Channels-last InstanceNorm (affine=False) with fused ReLU (HIP on GPU).

Drop-in for ``nn.InstanceNorm2d(C)`` as the reference encoders use it
(core/extractor.py, norm_fn='instance': no affine parameters, no running
statistics, so the module has no state_dict entries and checkpoints are
unaffected).  ``forward(x, relu=True)`` fuses the ReLU that always follows it.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ops, use_native


class _InstanceNormNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, relu: bool, eps: float):
        x = x.contiguous(memory_format=torch.channels_last)
        y, stats = ops().instance_norm_fwd(x, relu, eps)
        ctx.save_for_backward(x, stats)
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, stats = ctx.saved_tensors
        return ops().instance_norm_bwd(x, dy, stats, ctx.relu), None, None


class InstanceNorm2dNHWC(nn.Module):
    def __init__(self, num_features: int, eps: float = 1e-5):
        super().__init__()
        self.num_features = num_features
        self.eps = eps

    def forward(self, x: torch.Tensor, relu: bool = False) -> torch.Tensor:
        if (use_native(x) and x.dtype in (torch.bfloat16, torch.float32) and x.shape[1] % 8 == 0
                and x.is_contiguous(memory_format=torch.channels_last)):
            return _InstanceNormNHWC.apply(x, relu, self.eps)
        y = F.instance_norm(x, eps=self.eps)
        return F.relu(y) if relu else y

    def extra_repr(self) -> str:
        return f"{self.num_features}, eps={self.eps}, affine=False"
