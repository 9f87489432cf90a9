#!/usr/bin/env python3
"""fp32 inference paths after training: native split-bf16 encoders / update block vs the
module path, on a model trained a few fp32 steps (BatchNorm running statistics, weights
moved away from the init).

    python scripts/debug_split_eval.py --steps 60
"""
from __future__ import annotations

import argparse
import os
import sys
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--image_size", type=int, nargs=2, default=[256, 320])
    args = ap.parse_args()
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.optim import fetch_optimizer

    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    margs = Namespace(small=False, mixed_precision=False, amp_dtype="bf16", dropout=0.0, channels_last=True)
    model = RAFT(margs).to(dev).to(memory_format=torch.channels_last)
    opt, sched = fetch_optimizer(Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=args.steps), model)
    H, W = args.image_size
    i1, i2, flow, valid = synthetic_batch(1, H, W, max_disp=20.0, seed=10_000_000, device=dev)

    def run(native_encoder, fused_update):
        margs.native_encoder, margs.fused_update = native_encoder, fused_update
        model.eval()
        with torch.no_grad():
            low, up = model(i1, i2, iters=12, test_mode=True)
        model.train()
        margs.native_encoder = margs.fused_update = True
        return low.float(), up.float()

    def report(tag):
        ref_low, ref_up = run(False, False)
        gt = torch.sum((ref_up - flow) ** 2, dim=1).sqrt().mean().item()
        print(f"[{tag}] module path EPE vs gt {gt:.4f}", flush=True)
        for ne, fu in ((True, True), (True, False), (False, True)):
            low, up = run(ne, fu)
            d = torch.sum((up - ref_up) ** 2, dim=1).sqrt().mean().item()
            dl = torch.sum((low - ref_low) ** 2, dim=1).sqrt().mean().item()
            print(f"[{tag}] native_encoder={ne} fused_update={fu}: EPE vs module up {d:.5f} low {dl:.5f}",
                  flush=True)

    report("init")
    model.train()
    for step in range(args.steps):
        a, b, f, v = synthetic_batch(2, H, W, max_disp=20.0, seed=7 + step, device=dev)
        opt.zero_grad(set_to_none=True)
        loss, _ = sequence_loss(model(a, b, iters=12), f, v, 0.8)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()
    report(f"after {args.steps} steps")
    bn = [m for m in model.cnet.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    print("cnet BN running_mean |max|", max(m.running_mean.abs().max().item() for m in bn),
          "running_var range", min(m.running_var.min().item() for m in bn), max(m.running_var.max().item() for m in bn))


if __name__ == "__main__":
    main()
