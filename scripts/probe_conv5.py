#!/usr/bin/env python3
"""What bounds a conv_fwd5 step: the 128x128 / 8-wave tile as built (cfg 25), without its
MFMAs (30), without its DMA (31) and without either (32), on the update-block shapes; and
the fixed (per launch) vs per-step cost over a K sweep.

    python scripts/probe_conv5.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops import conv as C  # noqa: E402
from scripts.bench_convs import SHAPES, timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, H, W = 8, 46, 62
    P = B * H * W
    for name in ("conv", "q", "q15", "zr51", "convc2", "heads"):
        segs, cout, kh, kw = SHAPES[name]
        cin = sum(r for r, _ in segs)
        cin_p = sum(p for _, p in segs)
        x = torch.randn(P, cin_p, device=dev).bfloat16()
        w = torch.randn(cout, cin, kh, kw, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        wt = C.pack_fwd(w, segs)
        out = torch.empty(P, (cout + 7) // 8 * 8, device=dev, dtype=torch.bfloat16)
        g = C.geom(B, H, W, kh, kw, kh // 2, kw // 2)
        macs = P * cout * cin * kh * kw
        line = [f"{name:7s} N={cout:4d} K={cin * kh * kw:5d} steps={cin // 64 * kh * kw:3d}"]
        for cfg, tag in ((25, "full"), (30, "noMFMA"), (31, "noDMA"), (32, "neither")):
            us = timeit(lambda: C.conv_fwd([x], wt, g, cout, out[:, :cout], bias=b, act=1, cfg=cfg))
            line.append(f"{tag} {us:6.1f}us" + (f" ({2 * macs / us / 1e6:4.0f}TF)" if cfg == 25 else ""))
        print("  ".join(line), flush=True)
    # fixed vs per-step cost: the 3x3 N=128 conv over 1..8 input chunks of 64 channels
    for nck in (1, 2, 4, 8):
        cin = 64 * nck
        x = torch.randn(P, cin, device=dev).bfloat16()
        w = torch.randn(128, cin, 3, 3, device=dev) * 0.05
        b = torch.randn(128, device=dev)
        wt = C.pack_fwd(w, [(cin, cin)])
        out = torch.empty(P, 128, device=dev, dtype=torch.bfloat16)
        g = C.geom(B, H, W, 3, 3, 1, 1)
        line = [f"3x3 Cin={cin:4d} steps={9 * nck:3d}"]
        for cfg, tag in ((25, "full"), (30, "noMFMA"), (31, "noDMA"), (32, "neither")):
            us = timeit(lambda: C.conv_fwd([x], wt, g, 128, out, bias=b, act=1, cfg=cfg))
            line.append(f"{tag} {us:6.1f}us")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
