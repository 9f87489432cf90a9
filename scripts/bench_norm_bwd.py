#!/usr/bin/env python3
"""Norm-backward passes of the native encoders at the training shapes (config #2): the
reduce / finalize / apply kernels of enc_norm_bwd, per layer shape.
    python scripts/bench_norm_bwd.py        (RAFT_NORM_R / RAFT_NORM_PIX: chunking experiments)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops._ext import ops  # noqa: E402

SHAPES = [("fnet s1", 16, 184, 248, 64, 1), ("fnet s2", 16, 92, 124, 96, 1), ("fnet s3", 16, 46, 62, 128, 1),
          ("cnet s1", 8, 184, 248, 64, 2), ("cnet s2", 8, 92, 124, 96, 2), ("cnet s3", 8, 46, 62, 128, 2)]


def main():
    dev = torch.device("cuda")
    tot = 0.0
    for name, B, H, W, N, kind in SHAPES:
        g = torch.randn(B, H, W, N, device=dev).bfloat16()
        a0 = torch.randn(B, H, W, N, device=dev).bfloat16()
        c0 = torch.randn(B, 4, N, device=dev).abs()
        for _ in range(3):
            ops().enc_norm_bwd(g, a0, c0, True, None, None, kind)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            ops().enc_norm_bwd(g, a0, c0, True, None, None, kind)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1000
        tot += us
        gb = 5 * g.numel() * 2 / 1e9
        print(f"{name}: {B}x{H}x{W}x{N} kind {kind}: {us:6.1f} us for reduce+finalize+apply "
              f"({gb / us * 1e6 / 1e3:.2f} TB/s g, a0 read twice, da written)", flush=True)
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
