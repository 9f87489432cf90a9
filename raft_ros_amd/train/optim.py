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


def fetch_optimizer(args, model, capturable: bool = False, clip: float | None = None):
    """``capturable=True`` (GPU): lr lives in a device tensor and the step counter on the
    device, so the optimizer step can be captured in a HIP graph
    (``runtime.GraphedTrainStep``); the scheduler updates the lr tensor in place.

    ``clip`` (eager GPU training without a GradScaler): the native clip + AdamW step
    (ops/optim.py ``ClipAdamW``: clip_grad_norm_(clip) and AdamW in two launches, ~2.5 ms less
    host time per step); its ``step(skipped=...)`` clips, and returns the gradient norm."""
    params = [p for p in model.parameters() if p.requires_grad]
    if clip is not None and not capturable:
        from ..ops.optim import ClipAdamW, usable

        if usable(params):
            optimizer = ClipAdamW(params, lr=args.lr, weight_decay=args.wdecay, eps=args.epsilon, max_norm=float(clip))
            scheduler = optim.lr_scheduler.OneCycleLR(optimizer, args.lr, args.num_steps + 100, pct_start=0.05,
                                                      cycle_momentum=False, anneal_strategy="linear")
            return optimizer, scheduler
    fused = bool(params) and params[0].is_cuda
    capturable = capturable and fused
    lr = torch.tensor(float(args.lr), device=params[0].device) if capturable else args.lr
    kw = dict(lr=lr, weight_decay=args.wdecay, eps=args.epsilon)
    if capturable:
        kw["capturable"] = True
    try:
        optimizer = optim.AdamW(params, fused=fused, **kw)
    except (RuntimeError, TypeError):  # pragma: no cover - fused unsupported
        optimizer = optim.AdamW(params, **kw)
    scheduler = optim.lr_scheduler.OneCycleLR(optimizer, args.lr, args.num_steps + 100, pct_start=0.05,
                                              cycle_momentum=False, anneal_strategy="linear")
    return optimizer, scheduler
