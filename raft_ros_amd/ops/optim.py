"""Gradient clipping + AdamW as ONE native op (two HIP launches): the reference's optimizer step
(train.py:75-86 ``AdamW(lr, weight_decay, eps)``, train.py:154-157 ``clip_grad_norm_(..., clip)``).

torch's eager clip_grad_norm_ + fused AdamW cost ~2.6 ms of host time per training step on
MI355X (profiles/r5o_host_lead.log: clip 1.5 ms, optimizer 1.1 ms) for ~0.3 ms of GPU work --
at batch 1-2 per GPU (the per-rank work of train_standard.sh on 8 GPUs) the step is host-bound,
so that host time is step time.  ``ClipAdamW.step()`` validates the gradients and issues the two
kernels of csrc/optim.hip from C++ (~0.05 ms of host time):

  * the global gradient norm from fixed-order per-chunk partial sums (deterministic);
  * clip coefficient ``min(1, max_norm / (norm + 1e-6))`` (clip_grad_norm_'s);
  * a non-finite norm skips the update and the step count (the trainer's failure guard; like the
    fused AdamW's ``found_inf``) and adds 1 to ``skipped``;
  * the AdamW update of torch's fused kernel: decoupled decay ``p *= 1 - lr * wd``, moments,
    bias corrections, ``p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)``.

The state dict has torch AdamW's layout (``exp_avg``, ``exp_avg_sq``, ``step`` per parameter),
so checkpoints and resume sidecars are interchangeable with ``torch.optim.AdamW``.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import ops

CHUNK = 16384  # csrc/kernel_abi.h kAdamChunk


class ClipAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 max_norm: float = 0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, max_norm=max_norm))
        if len(self.param_groups) != 1:
            raise ValueError("ClipAdamW: one parameter group (the reference's optimizer)")
        self._plan = None
        self._steps: Optional[torch.Tensor] = None
        self._par = 0

    # ------------------------------------------------------------------ tables
    def _build(self):
        params = [p for p in self.param_groups[0]["params"] if p.requires_grad]
        dev = params[0].device
        ptrs, blocks, tblk = [], [], [0]
        for i, p in enumerate(params):
            if p.dtype != torch.float32 or not p.is_cuda:
                raise ValueError("ClipAdamW: fp32 GPU parameters")
            st = self.state[p]
            if "exp_avg" not in st:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            for t in (st["exp_avg"], st["exp_avg_sq"]):
                if t.stride() != p.stride() or t.dtype != torch.float32:
                    raise ValueError("ClipAdamW: moments must share the parameter's layout")
            ptrs += [p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()]
            n = p.numel()
            for s0 in range(0, n, CHUNK):
                blocks += [i, s0, min(CHUNK, n - s0)]
            tblk.append(len(blocks) // 3)
        step0 = 0.0
        for p in params:
            s = self.state[p].get("step")
            if s is not None:
                step0 = float(s)
                break
        if self._steps is None:
            self._steps = torch.zeros(2, device=dev)
        self._steps.fill_(step0)
        self._par = 0
        self._plan = (params, torch.tensor(ptrs, dtype=torch.int64, device=dev),
                      torch.tensor(blocks, dtype=torch.int32, device=dev), tblk,
                      torch.empty(tblk[-1], device=dev))
        self.norm = torch.zeros((), device=dev)

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, closure=None, skipped: Optional[torch.Tensor] = None):
        """Clip the gradients to ``max_norm`` (0: no clipping) and take one AdamW step; returns
        the total gradient norm (a device tensor, before clipping)."""
        loss = closure() if closure is not None else None
        if self._plan is None:
            self._build()
        params, ptrs, blocks, tblk, partial = self._plan
        grads = [p.grad for p in params]
        if any(g is None for g in grads):
            raise RuntimeError("ClipAdamW: every parameter needs a gradient (RAFT trains all of them)")
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        ops().clip_adamw_(params, grads, ptrs, blocks, tblk, partial, self._steps, self._par, float(g["lr"]),
                          float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), float(g["max_norm"]),
                          self.norm, skipped)
        self._par ^= 1
        return self.norm if closure is None else loss

    # ------------------------------------------------------------------ state dict (torch AdamW layout)
    def state_dict(self):
        if self._plan is not None:
            step = self._steps[self._par].detach().clone()
            for p in self._plan[0]:
                self.state[p]["step"] = step.clone()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for st in self.state.values():  # torch AdamW's per-parameter fp32 step tensors
            if "step" in st and torch.is_tensor(st["step"]):
                st["step"] = st["step"].float()
        self._plan = None  # new moment tensors: rebuild the pointer tables (and the step slots)


def usable(params) -> bool:
    """The native step applies: fp32 parameters on the GPU with the extension loaded."""
    from ._ext import is_loaded

    ps = [p for p in params if p.requires_grad]
    return bool(ps) and all(p.is_cuda and p.dtype == torch.float32 for p in ps) and is_loaded()
