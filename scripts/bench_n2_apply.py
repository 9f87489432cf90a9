#!/usr/bin/env python3
"""n2_apply (flow_head.conv2 from the heads conv's per-tap partials + the coordinate update)
per launch at the config #2 and 1080p shapes.  python scripts/bench_n2_apply.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops._ext import ops  # noqa: E402
from scripts.bench_convs import timeit  # noqa: E402


def main():
    k = ops()
    for name, (B, H, W) in {"train 8x46x62": (8, 46, 62), "1080p 1x135x240": (1, 135, 240)}.items():
        P = B * H * W
        y = torch.randn(4, 18, P, device="cuda")
        bias = torch.randn(2, device="cuda")
        c1 = torch.randn(B, 2, H, W, device="cuda")
        co, fl = torch.empty_like(c1), torch.empty_like(c1)
        us = timeit(lambda: k.n2_apply(y, bias, c1, co, fl, None))
        print(f"{name:18s} n2_apply {us:7.2f} us  ({4 * 18 * P * 4 / us / 1e3:6.0f} GB/s of partials)")


if __name__ == "__main__":
    main()
