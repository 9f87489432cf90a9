#!/usr/bin/env python3
"""Correlation-volume GEMM timing (the dense pyramid build, ops/corr.py _BuildPyramid):
v2 store-oriented kernel vs the generic one (cfg=1), at the training and 1080p shapes.

    python scripts/bench_corr.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops._ext import ops  # noqa: E402


def ld_of(H, W, levels=4):
    return sum(-(-(W >> l) // 16) * 16 * (H >> l) for l in range(levels))


def main():
    dev = torch.device("cuda")
    k = ops()
    for name, B, H, W in (("train 8x368x496", 8, 46, 62), ("sintel 1x440x1024", 1, 55, 128), ("1080p", 1, 135, 240)):
        HW, ld, C = H * W, ld_of(H, W), 256
        A = torch.randn(B, HW, C, device=dev).bfloat16()
        Bm = torch.randn(B, ld, C, device=dev).bfloat16()
        out = torch.empty(B * HW, ld, device=dev, dtype=torch.bfloat16)
        line = [f"{name:18s} M={HW} N={ld} K={C} batch={B}"]
        for cfg in (0, 1):
            fn = lambda: k.corr_gemm(A, Bm, out, HW, ld, C, B, C, HW * C, C, ld * C, ld, HW * ld, 0.0625, False,  # noqa
                                     False, 0, cfg)
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / 10 * 1000
            tf = 2 * B * HW * ld * C / us / 1e6
            gbs = B * HW * ld * 2 / us / 1e3
            line.append(f"cfg{cfg}: {us:8.1f} us {tf:6.0f} TF/s  store {gbs:6.0f} GB/s")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
