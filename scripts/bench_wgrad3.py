#!/usr/bin/env python3
"""Batched 5-tap / 3x3 weight gradients of the refinement step (12 iterations of config #2, as
_PackWeights.backward runs them) against an fp32 torch reference: time per launch, TF/s and the
relative error of the weight / bias gradients.  Variants chosen by environment switches are A/B'd
as separate processes.

    python scripts/bench_wgrad3.py [--batch 8] [--hw 46 62] [--iters 12]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops import conv as C  # noqa: E402
from scripts.bench_convs import timeit  # noqa: E402

# name: (cin, cout, kh, kw)
SHAPES = {"zr15": (384, 256, 1, 5), "q15": (384, 128, 1, 5), "zr51": (384, 256, 5, 1), "q51": (384, 128, 5, 1),
          "conv33": (256, 126, 3, 3), "heads33": (128, 512, 3, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, nargs=2, default=[46, 62])
    ap.add_argument("--iters", type=int, default=12)
    args = ap.parse_args()
    dev = torch.device("cuda")
    B, (H, W), T = args.batch, args.hw, args.iters
    P = T * B * H * W
    torch.manual_seed(0)
    for name, (cin, cout, kh, kw) in SHAPES.items():
        x = (torch.randn(P, cin, device=dev) * 0.5).bfloat16()
        dy = (torch.randn(P, (cout + 7) // 8 * 8, device=dev) * 0.5).bfloat16()
        w = torch.empty(cout, cin, kh, kw, device=dev)
        b = torch.empty(cout, device=dev)
        g = C.geom(T * B, H, W, kh, kw, kh // 2, kw // 2)
        segs = [(cin, cin)]
        run = lambda: C.conv_wgrad_params([x], dy, g, [w], [b], segs)  # noqa: E731
        run()
        torch.cuda.synchronize()
        # fp32 reference on a few images (the reduction covers every pixel; check a slice)
        n = 2
        xi = x[:n * H * W].float().view(n, H, W, cin).permute(0, 3, 1, 2)
        gi = dy[:n * H * W, :cout].float().view(n, H, W, cout).permute(0, 3, 1, 2)
        ws = torch.empty_like(w)
        bs = torch.empty_like(b)
        C.conv_wgrad_params([x[:n * H * W]], dy[:n * H * W], C.geom(n, H, W, kh, kw, kh // 2, kw // 2), [ws],
                            [bs], segs)
        wr = torch.nn.grad.conv2d_weight(xi, w.shape, gi, padding=(kh // 2, kw // 2))
        err = ((ws - wr).norm() / wr.norm()).item()
        berr = ((bs - gi.sum((0, 2, 3))).norm() / gi.sum((0, 2, 3)).norm()).item()
        us = timeit(run, reps=10)
        flop = 2 * P * cout * cin * kh * kw
        print(f"{name:8s} cin={cin} cout={cout} {kh}x{kw}: {us:7.1f} us  {flop / us / 1e6:5.0f} TF/s  "
              f"rel err w {err:.2e} b {berr:.2e}", flush=True)


if __name__ == "__main__":
    main()
