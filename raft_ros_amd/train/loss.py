"""Sequence loss and flow metrics (reference train.py:42-72).

``loss = sum_i gamma^(n-i-1) * mean(valid * |pred_i - gt|)`` with
``valid = (valid >= 0.5) & (|gt| < max_flow)``; metrics (EPE, 1/3/5 px) over
valid pixels of the final prediction.  Unlike the reference, metrics stay on
the device (no four ``.item()`` host syncs per step); call
``metrics_to_host`` when logging.
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ..ops._ext import ops, use_native

MAX_FLOW = 400.0


class _FusedSeqLoss(torch.autograd.Function):
    """One HIP pass forward (loss + metric sums), one pass backward (all n
    prediction gradients); raft_ros_amd/csrc/seq_loss.hip."""

    @staticmethod
    def forward(ctx, flow_gt, valid, gamma, max_flow, *preds):
        sums = ops().seq_loss(list(preds), flow_gt, valid, gamma, max_flow)
        ctx.save_for_backward(flow_gt, valid, *preds)
        ctx.gamma, ctx.max_flow = gamma, max_flow
        ctx.mark_non_differentiable(sums)
        loss = sums[0] / float(2 * valid.numel())
        return loss, sums

    @staticmethod
    def backward(ctx, gloss, _gsums):
        flow_gt, valid, *preds = ctx.saved_tensors
        grads = ops().seq_loss_backward(preds, flow_gt, valid, gloss.float().reshape(1), ctx.gamma,
                                        ctx.max_flow)
        if grads and grads[0].is_cuda:
            # when the gradients are ready: the fused refinement steps start their upsampler /
            # head backward on a side stream from this event (ops/update_fused.py)
            ready = torch.cuda.Event()
            ready.record()
            for g in grads:
                g._raft_ready = ready
        return (None, None, None, None, *grads)


def _fused_ok(flow_preds, flow_gt) -> bool:
    return (use_native(flow_gt) and 1 <= len(flow_preds) <= 32 and flow_gt.dtype == torch.float32
            and all(p.dtype == torch.float32 and p.shape == flow_gt.shape for p in flow_preds))


METRIC_KEYS = ("epe", "1px", "3px", "5px")  # the metrics sequence_loss returns


def sequence_loss(flow_preds: List[torch.Tensor], flow_gt: torch.Tensor, valid: torch.Tensor,
                  gamma: float = 0.8, max_flow: float = MAX_FLOW):
    if _fused_ok(flow_preds, flow_gt):
        preds = [p.contiguous() for p in flow_preds]
        loss, s = _FusedSeqLoss.apply(flow_gt.contiguous(), valid.float().contiguous(), float(gamma),
                                      float(max_flow), *preds)
        cnt = s[5].clamp_min(1.0)
        return loss, {"epe": s[1] / cnt, "1px": s[2] / cnt, "3px": s[3] / cnt, "5px": s[4] / cnt}
    n = len(flow_preds)
    mag = torch.sum(flow_gt ** 2, dim=1).sqrt()
    valid = (valid >= 0.5) & (mag < max_flow)
    vmask = valid[:, None].to(flow_gt.dtype)
    loss = flow_gt.new_zeros(())
    for i, pred in enumerate(flow_preds):
        w = gamma ** (n - i - 1)
        loss = loss + w * (vmask * (pred - flow_gt).abs()).mean()
    # metrics carry no autograd graph (a live graph would pin the AccumulateGrad nodes)
    epe = torch.sum((flow_preds[-1].detach() - flow_gt) ** 2, dim=1).sqrt()
    vf = valid.to(epe.dtype)
    cnt = vf.sum().clamp_min(1.0)
    metrics = {
        "epe": (epe * vf).sum() / cnt,
        "1px": ((epe < 1).to(epe.dtype) * vf).sum() / cnt,
        "3px": ((epe < 3).to(epe.dtype) * vf).sum() / cnt,
        "5px": ((epe < 5).to(epe.dtype) * vf).sum() / cnt,
    }
    return loss, metrics


def metrics_to_host(metrics: Dict[str, torch.Tensor]) -> Dict[str, float]:
    if not metrics:
        return {}
    keys = sorted(metrics)
    vals = torch.stack([metrics[k].detach().float() for k in keys]).cpu().tolist()
    return dict(zip(keys, vals))
