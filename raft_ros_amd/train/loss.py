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

MAX_FLOW = 400.0


def sequence_loss(flow_preds: List[torch.Tensor], flow_gt: torch.Tensor, valid: torch.Tensor,
                  gamma: float = 0.8, max_flow: float = MAX_FLOW):
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
