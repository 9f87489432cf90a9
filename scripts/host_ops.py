#!/usr/bin/env python3
"""Where does the host spend the training step?  torch.profiler (CPU activity only) over
steady-state bench steps, once pipelined (the GPU busy behind the host) and once with the GPU
drained before every step: ops whose host time grows in the pipelined run block on the GPU.

    python scripts/host_ops.py [--steps 4] [--top 30]
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
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile

    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.optim import fetch_optimizer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", dropout=0.0)).to(dev)
    model = model.to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000), model)
    pool = [synthetic_batch(8, 368, 496, seed=i, device=dev) for i in range(4)]

    def step(i):
        i1, i2, flow, valid = pool[i % len(pool)]
        opt.zero_grad(set_to_none=True)
        loss, _ = sequence_loss(model(i1, i2, iters=12), flow, valid, gamma=0.8)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()

    for i in range(6):
        step(i)
    torch.cuda.synchronize()
    res = {}
    for mode in ("pipelined", "drained"):
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            for i in range(args.steps):
                if mode == "drained":
                    torch.cuda.synchronize()
                step(i)
            torch.cuda.synchronize()
        res[mode] = {e.key: e.self_cpu_time_total / args.steps for e in prof.key_averages()}
        tot = sum(res[mode].values())
        print(f"== {mode}: self CPU {tot / 1e3:.2f} ms/step")
    keys = sorted(res["pipelined"], key=lambda k: -(res["pipelined"][k] - res["drained"].get(k, 0.0)))
    print(f"{'op':60s} {'pipelined us':>13s} {'drained us':>11s}")
    for k in keys[:args.top]:
        print(f"{k[:60]:60s} {res['pipelined'][k]:13.1f} {res['drained'].get(k, 0.0):11.1f}")
    print("top ops by pipelined self CPU:")
    for k in sorted(res["pipelined"], key=lambda k: -res["pipelined"][k])[:args.top]:
        print(f"{k[:60]:60s} {res['pipelined'][k]:13.1f} {res['drained'].get(k, 0.0):11.1f}")


if __name__ == "__main__":
    main()
