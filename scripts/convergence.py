#!/usr/bin/env python3
"""Synthetic-data training convergence: native HIP path vs the reference op path.

Both runs train RAFT-base from the same random init (seed) on the same stream of
synthetic pairs (textures warped by known smooth flows, exact ground truth;
``data/synthetic.py``) with the reference training recipe (sequence loss
gamma 0.8, AdamW, OneCycle, clip 1.0, 12 iterations; train.py:47-86) and
evaluate the same held-out synthetic pairs every ``--eval_every`` steps
(test_mode, 12 iterations, EPE over valid pixels).  ``--impl reference``
swaps every native op for the reference's PyTorch op sequence (grid_sample
lookup, dense fp32 matmul volume, MIOpen convs), so the two curves isolate
the numerics of the MI355X kernels.  One JSON line per evaluation.

    python scripts/convergence.py --impl native --steps 2000 > native.jsonl
    python scripts/convergence.py --impl reference --steps 2000 > reference.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", choices=["native", "reference"], default="native")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--image_size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--lr", type=float, default=4e-4)
    ap.add_argument("--eval_every", type=int, default=100)
    ap.add_argument("--eval_pairs", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--max_disp", type=float, default=20.0)
    ap.add_argument("--precision", choices=["bf16", "fp32"], default="bf16",
                    help="fp32: no autocast (the reference's train_standard.sh recipe); bf16: AMP")
    args = ap.parse_args()

    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.ops import _ext
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.optim import fetch_optimizer

    dev = torch.device("cuda", 0)
    _ext.set_backend(args.impl)
    torch.manual_seed(args.seed)
    model = RAFT(Namespace(small=False, mixed_precision=args.precision == "bf16", amp_dtype="bf16", dropout=0.0,
                           channels_last=args.impl == "native")).to(dev)
    if args.impl == "native":
        model = model.to(memory_format=torch.channels_last)
    opt, sched = fetch_optimizer(Namespace(lr=args.lr, wdecay=1e-4, epsilon=1e-8, num_steps=args.steps), model)
    H, W = args.image_size
    evalset = [synthetic_batch(1, H, W, max_disp=args.max_disp, seed=10_000_000 + i, device=dev)
               for i in range(args.eval_pairs)]

    def evaluate():
        model.eval()
        tot = cnt = 0.0
        with torch.no_grad():
            for i1, i2, flow, valid in evalset:
                _, up = model(i1, i2, iters=args.iters, test_mode=True)
                epe = torch.sum((up.float() - flow) ** 2, dim=1).sqrt()[valid >= 0.5]
                tot += epe.sum().item()
                cnt += epe.numel()
        model.train()
        return tot / max(cnt, 1.0)

    t0 = time.perf_counter()
    model.train()
    for step in range(args.steps + 1):
        if step % args.eval_every == 0:
            rec = {"impl": args.impl, "precision": args.precision, "step": step, "val_epe": round(evaluate(), 5),
                   "elapsed_s": round(time.perf_counter() - t0, 1)}
            print(json.dumps(rec), flush=True)
        if step == args.steps:
            break
        i1, i2, flow, valid = synthetic_batch(args.batch, H, W, max_disp=args.max_disp, seed=args.seed * 7919 + step,
                                              device=dev)
        opt.zero_grad(set_to_none=True)
        loss, metrics = sequence_loss(model(i1, i2, iters=args.iters), flow, valid, 0.8)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()
        if step % 50 == 0:
            print(json.dumps({"impl": args.impl, "precision": args.precision, "step": step, "loss": round(loss.item(), 4),
                              "train_epe": round(metrics["epe"].item(), 4)}), flush=True)


if __name__ == "__main__":
    main()
