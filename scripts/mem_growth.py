#!/usr/bin/env python3
"""Does device memory grow across training steps?  Per step: allocated / reserved bytes and
the number of live refinement-run objects (ops/update_fused._Run) still reachable, with and
without a gc.collect() after each step.

    python scripts/mem_growth.py [--steps 12] [--batch 8] [--collect]
"""
from __future__ import annotations

import argparse
import gc
import os
import sys
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--image_size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--collect", action="store_true")
    args = ap.parse_args()
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.ops import update_fused as uf
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.optim import fetch_optimizer

    dev = torch.device("cuda", 0)
    model = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", dropout=0.0)).to(dev)
    model = model.to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000), model, clip=1.0)
    pool = [synthetic_batch(args.batch, *args.image_size, seed=i, device=dev) for i in range(4)]
    for i in range(args.steps):
        i1, i2, flow, valid = pool[i % 4]
        opt.zero_grad(set_to_none=True)
        preds = model(i1, i2, iters=12)
        loss, _ = sequence_loss(preds, flow, valid, gamma=0.8)
        loss.backward()
        opt.step()
        sched.step()
        del preds, loss
        torch.cuda.synchronize()
        if args.collect:
            gc.collect()
        runs = sum(1 for o in gc.get_objects() if isinstance(o, uf._Run))
        print(f"step {i:3d}  allocated {torch.cuda.memory_allocated(dev) / 2**20:8.1f} MiB  reserved "
              f"{torch.cuda.memory_reserved(dev) / 2**20:8.1f} MiB  live _Run {runs}  gc counts {gc.get_count()}",
              flush=True)
    if not args.collect:
        n = gc.collect()
        runs = sum(1 for o in gc.get_objects() if isinstance(o, uf._Run))
        print(f"after gc.collect() ({n} objects): allocated {torch.cuda.memory_allocated(dev) / 2**20:8.1f} MiB  "
              f"live _Run {runs}", flush=True)


if __name__ == "__main__":
    main()
