#!/usr/bin/env python3
"""Host-issue vs GPU time per training-step phase (RAFT-base, bench config #2).

For each phase (forward, loss, backward, clip, optimizer) the GPU is drained first,
then the phase is issued: ``issue`` is the host time until the Python call returns,
``gpu`` the time until the GPU has finished it.  issue > gpu means that phase is
host-bound (the GPU idles while kernels are being launched).
Usage: python scripts/cpu_issue.py [--steps 5]"""
import argparse
import os
import sys
import time
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    args = ap.parse_args()
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.optim import fetch_optimizer

    dev = torch.device("cuda", 0)
    model = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", dropout=0.0,
                           channels_last=True, fused_update=True)).to(dev).to(memory_format=torch.channels_last)
    model.train()
    opt, sched = fetch_optimizer(Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000), model)
    i1, i2, flow, valid = synthetic_batch(args.batch, 368, 496, seed=0, device=dev)
    tot = {}

    def phase(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        tot.setdefault(name, []).append(((t1 - t0) * 1e3, (t2 - t0) * 1e3))
        return out

    for it in range(args.steps + 2):
        opt.zero_grad(set_to_none=True)
        preds = phase("forward", lambda: model(i1, i2, iters=12))
        loss, _ = phase("loss", lambda: sequence_loss(preds, flow, valid, gamma=0.8))
        phase("backward", lambda: loss.backward())
        phase("clip", lambda: torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0))
        phase("optimizer", lambda: (opt.step(), sched.step()))
        if it == 1:
            tot.clear()
    for k, v in tot.items():
        iss = sum(a for a, _ in v) / len(v)
        gpu = sum(b for _, b in v) / len(v)
        print(f"{k:10s} issue {iss:8.3f} ms   issue+drain {gpu:8.3f} ms   {'HOST-BOUND' if iss > 0.9 * gpu else ''}")


if __name__ == "__main__":
    main()
