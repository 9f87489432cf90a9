"""Opt-in synchronized BatchNorm for the context encoder under DDP (``train.py --sync_bn``).

The reference trains with single-process ``nn.DataParallel`` (train.py:138), whose replicas
each normalise with the statistics of their own slice of the batch; per-rank BatchNorm is
therefore the default here too.  The chairs stage, however, trains the context encoder's
BatchNorm (core/raft.py:55) at a global batch of 10, which over 8 ranks leaves 1-2 images
per replica.  ``--sync_bn`` makes every rank normalise with the statistics of the WHOLE
global batch instead:

* :class:`SyncBatchNorm2d` is an ``nn.BatchNorm2d`` (same parameters, buffers and
  ``state_dict`` keys, so ``raft-*.pth`` checkpoints are unchanged) whose training-mode
  forward all-reduces (count, sum, sum of squares) and whose backward all-reduces
  (sum dy, sum dy * xhat) over the process group -- one small collective each way per
  norm layer, over RCCL (xGMI) on the GPU or gloo on the CPU;
* on the GPU the native encoder kernels (ops/encoder.py) do the same with their own
  statistics: the per-tile (sum, M2) conv-epilogue statistics are all-gathered before the
  finalize kernel, and the norm backward's partial sums are all-gathered between its
  reduce and finalize passes (``enc_norm_bwd_part`` / ``enc_norm_bwd_finish``).

Running statistics are updated from the global statistics on every rank, so they stay
identical across ranks.  Parameter gradients (weight, bias) stay per-rank sums, which DDP
then averages like every other gradient -- the combination equals the gradient of the
full-batch loss.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def group_size(group) -> int:
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def is_synced(m: nn.Module) -> bool:
    """True when ``m`` normalises over the process group in its current mode."""
    return isinstance(m, SyncBatchNorm2d) and m.training and group_size(m.process_group) > 1


def all_gather_cat(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate every rank's ``t`` (same shape everywhere) along dim 0, rank-major."""
    n = group_size(group)
    if n == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(n)]
    dist.all_gather(parts, t.contiguous(), group=group)
    return torch.cat(parts, 0)


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, group):
        xf = x.float()
        dims = [0, 2, 3]
        C = x.shape[1]
        # per-rank (count, mean, M2) gathered and Chan-combined: no E[x^2] - E[x]^2 cancellation
        cnt = float(x.numel() // C)
        lmean = xf.mean(dims)
        lm2 = ((xf - lmean.view(1, C, 1, 1)) ** 2).sum(dims)
        st = all_gather_cat(torch.cat([torch.full((1,), cnt, device=x.device), lmean, lm2])[None], group)
        ns, means, m2s = st[:, :1], st[:, 1:1 + C], st[:, 1 + C:]
        n = ns.sum()
        mean = (ns * means).sum(0) / n
        var = (m2s.sum(0) + (ns * (means - mean) ** 2).sum(0)) / n
        invstd = torch.rsqrt(var + eps)
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
                unbiased = var * (n / (n - 1).clamp_min(1.0))
                running_var.mul_(1 - momentum).add_(unbiased.to(running_var.dtype), alpha=momentum)
        xhat = (xf - mean.view(1, C, 1, 1)) * invstd.view(1, C, 1, 1)
        w = weight.float() if weight is not None else torch.ones_like(mean)
        b = bias.float() if bias is not None else torch.zeros_like(mean)
        y = xhat * w.view(1, C, 1, 1) + b.view(1, C, 1, 1)
        ctx.save_for_backward(xhat, invstd, w, n.reshape(1))
        ctx.group = group
        ctx.has_w, ctx.has_b = weight is not None, bias is not None
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, gy):
        xhat, invstd, w, n = ctx.saved_tensors
        C = xhat.shape[1]
        g = gy.float()
        dims = [0, 2, 3]
        sum_dy = g.sum(dims)
        sum_dy_xhat = (g * xhat).sum(dims)
        glob = torch.cat([sum_dy, sum_dy_xhat])
        dist.all_reduce(glob, group=ctx.group)
        gdy, gdyx = glob[:C] / n, glob[C:] / n
        dx = (g - gdy.view(1, C, 1, 1) - xhat * gdyx.view(1, C, 1, 1)) * (w * invstd).view(1, C, 1, 1)
        dw = sum_dy_xhat if ctx.has_w else None  # per-rank sums: DDP averages them
        db = sum_dy if ctx.has_b else None
        return dx.to(gy.dtype), dw, db, None, None, None, None, None


class SyncBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` that normalises over the process group in training mode (see the
    module docstring).  Outside a process group, or in eval mode, it is a plain BatchNorm."""

    def __init__(self, *args, process_group=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.process_group = process_group

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not (self.training and group_size(self.process_group) > 1):
            return super().forward(x)
        if self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
        momentum = self.momentum
        if momentum is None:  # cumulative moving average, as nn.BatchNorm2d
            momentum = 1.0 / float(self.num_batches_tracked)
        rm = self.running_mean if self.track_running_stats else None
        rv = self.running_var if self.track_running_stats else None
        return _SyncBNFn.apply(x, self.weight, self.bias, rm, rv, self.eps, momentum, self.process_group)


def convert_sync_bn(module: nn.Module, process_group=None, _memo=None) -> nn.Module:
    """Replace every ``nn.BatchNorm2d`` under ``module`` by a :class:`SyncBatchNorm2d` that
    shares its parameters and buffers (in place; returns ``module``).  A norm reachable under
    two names (a residual block's ``norm3`` is also ``downsample[1]``) becomes ONE module."""
    memo = {} if _memo is None else _memo
    for name, child in list(module.named_children()):
        if isinstance(child, nn.BatchNorm2d) and not isinstance(child, SyncBatchNorm2d):
            new = memo.get(id(child))
            if new is None:
                new = SyncBatchNorm2d(child.num_features, eps=child.eps, momentum=child.momentum,
                                      affine=child.affine, track_running_stats=child.track_running_stats,
                                      process_group=process_group)
                new.weight, new.bias = child.weight, child.bias
                if child.track_running_stats:
                    new.running_mean, new.running_var = child.running_mean, child.running_var
                    new.num_batches_tracked = child.num_batches_tracked
                new.train(child.training)
                memo[id(child)] = new
            setattr(module, name, new)
        else:
            convert_sync_bn(child, process_group, memo)
    return module


def native_norm_stats(st: torch.Tensor, group) -> tuple:
    """Synchronized-BN forward helper of the native encoder: every rank's per-tile conv
    statistics (sum, M2), gathered rank-major.  Returns (stats of all ranks, image count)."""
    allst = all_gather_cat(st, group)
    return allst, allst.shape[0]


def native_norm_bwd(o, g, a0, c0, relu0, a1, c1, kind, group, split: bool = False):
    """Synchronized-BN backward of the native encoder's norm tail: reduce pass per rank,
    all-gather of the partial sums, finalize over the global batch, apply per rank.  The
    returned dgamma / dbeta are this rank's own sums (DDP averages them)."""
    part = o.enc_norm_bwd_part(g, a0, c0, relu0, a1, c1, kind, split)
    allp = all_gather_cat(part, group)
    r = list(o.enc_norm_bwd_finish(g, a0, c0, relu0, a1, c1, kind, allp, allp.shape[0], split))
    loc = part.sum((0, 1))  # [4, N]: dbeta0, dgamma0, dbeta1, dgamma1 of this rank
    r[2], r[3] = loc[1].contiguous(), loc[0].contiguous()
    if a1 is not None:
        r[4], r[5] = loc[3].contiguous(), loc[2].contiguous()
    return r
