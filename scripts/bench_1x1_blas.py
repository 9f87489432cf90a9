#!/usr/bin/env python3
"""The update block's 1x1 convs (config #2: 8 x 46 x 62 pixels) as plain GEMMs: the
hand-written implicit-GEMM forward (auto choice: v4 64x128) vs hipBLASLt through torch
(mm / addmm with bias, + relu), same bf16 operands.

    python scripts/bench_1x1_blas.py [--batch 8] [--hw 46 62]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops import conv as C  # noqa: E402
from scripts.bench_convs import timeit  # noqa: E402

SHAPES = {"convc1": (384, 256), "mask2": (256, 576), "d_convc1": (256, 384), "d_mask2": (576, 256)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, nargs=2, default=[46, 62])
    args = ap.parse_args()
    dev = torch.device("cuda")
    B, (H, W) = args.batch, args.hw
    P = B * H * W
    for name, (cin, cout) in SHAPES.items():
        x = torch.randn(P, cin, device=dev).bfloat16()
        w = torch.randn(cout, cin, 1, 1, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        wt = C.pack_fwd(w)
        g = C.geom(B, H, W, 1, 1, 0, 0)
        out = torch.empty(P, cout, device=dev, dtype=torch.bfloat16)
        wT = w.view(cout, cin).t().bfloat16().contiguous()
        bb = b.bfloat16()
        t_ours = timeit(lambda: C.conv_fwd([x], wt, g, cout, out, bias=b, act=1, cfg=0))
        t_mm = timeit(lambda: torch.mm(x, wT))
        t_addmm = timeit(lambda: torch.addmm(bb, x, wT))
        t_relu = timeit(lambda: torch._addmm_activation(bb, x, wT))
        flops = 2 * P * cin * cout
        ref = torch.relu(torch.addmm(bb, x, wT))
        C.conv_fwd([x], wt, g, cout, out, bias=b, act=1, cfg=0)
        err = float((out.float() - ref.float()).abs().max())
        print(f"{name:9s} P={P} K={cin} N={cout}: ours {t_ours:6.1f} us ({flops / t_ours / 1e6:4.0f} TF) | "
              f"mm {t_mm:6.1f} | addmm {t_addmm:6.1f} | addmm+relu {t_relu:6.1f} us | max diff {err:.3f}",
              flush=True)


if __name__ == "__main__":
    main()
