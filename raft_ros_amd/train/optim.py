"""Optimizer + LR schedule (reference train.py:75-86).

AdamW(lr, weight_decay, eps) and OneCycleLR(max_lr=lr, total_steps=num_steps+100,
pct_start=0.05, cycle_momentum=False, anneal_strategy='linear').  On GPU the
fused AdamW implementation is used (one multi-tensor launch per step).
"""
from __future__ import annotations

import torch
import torch.optim as optim


def count_parameters(model) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def fetch_optimizer(args, model):
    params = [p for p in model.parameters() if p.requires_grad]
    kw = dict(lr=args.lr, weight_decay=args.wdecay, eps=args.epsilon)
    fused = bool(params) and params[0].is_cuda
    try:
        optimizer = optim.AdamW(params, fused=fused, **kw)
    except (RuntimeError, TypeError):  # pragma: no cover - fused unsupported
        optimizer = optim.AdamW(params, **kw)
    scheduler = optim.lr_scheduler.OneCycleLR(optimizer, args.lr, args.num_steps + 100, pct_start=0.05,
                                              cycle_momentum=False, anneal_strategy="linear")
    return optimizer, scheduler
