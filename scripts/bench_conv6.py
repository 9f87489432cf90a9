#!/usr/bin/env python3
"""conv_fwd6 (lean halo strip) vs the automatic choice (v5 / v4) on the update-block conv
shapes at config #2 (8 x 46 x 62 pixels): bitwise / numeric agreement and time per launch.

    python scripts/bench_conv6.py [--cfgs 41,45,59,60] [--batch 8] [--hw 46 62]
cfg 41 = 256x64 flat strip, 45 = 256x128 flat strip, 59 / 60 = 256x64 as 2-D 4x64 / 8x32 tiles,
62-65 = 128x64 2-D / flat tiles (two workgroups per CU), 74 / 75 = 64x64 2-D tiles (three per CU).
(The probe variants behind profiles/r3_conv6_probe.log -- no MFMA / DMA / reads / barrier /
epilogue -- were removed after the measurement.)
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

# name: (cin, cout, kh, kw) -- forward convs and the data-gradient shapes (Cin = fwd N)
SHAPES = {
    "conv": (256, 126, 3, 3),
    "convc2": (256, 192, 3, 3),
    "convf2": (128, 64, 3, 3),
    "heads": (128, 512, 3, 3),
    "fh1": (128, 256, 3, 3),
    "fh2": (256, 2, 3, 3),
    "zr": (384, 256, 1, 5),
    "q15": (384, 128, 1, 5),
    "zr51": (384, 256, 5, 1),
    "q51": (384, 128, 5, 1),
    "d_conv": (128, 256, 3, 3),
    "d_convc2": (192, 256, 3, 3),
    "d_fh1": (256, 128, 3, 3),
    "d_zr15": (256, 384, 1, 5),
    "d_q15": (128, 384, 1, 5),
    "d_zr51": (256, 384, 5, 1),
    "d_q51": (128, 384, 5, 1),
    "convc1": (384, 256, 1, 1),
    "mask2": (256, 576, 1, 1),
    "d_convc1": (256, 384, 1, 1),
    "d_mask2": (576, 256, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="62,63,64,65,74,75")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, nargs=2, default=[46, 62])
    ap.add_argument("--only", default="")

    args = ap.parse_args()
    dev = torch.device("cuda")
    B, (H, W) = args.batch, args.hw
    P = B * H * W
    cfgs = [int(c) for c in args.cfgs.split(",")]
    names = args.only.split(",") if args.only else list(SHAPES)
    torch.manual_seed(0)
    for name in names:
        cin, cout, kh, kw = SHAPES[name]
        x = torch.randn(P, cin, device=dev).bfloat16()
        w = torch.randn(cout, cin, kh, kw, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        wt = C.pack_fwd(w)
        g = C.geom(B, H, W, kh, kw, kh // 2, kw // 2)
        cp = (cout + 7) // 8 * 8
        macs = P * cout * cin * kh * kw
        ref_out = torch.zeros(P, cp, device=dev, dtype=torch.bfloat16)
        C.conv_fwd([x], wt, g, cout, ref_out[:, :cout], bias=b, act=1, cfg=0)
        # fp32 torch oracle
        xi = x.float().view(B, H, W, cin).permute(0, 3, 1, 2)
        yt = F.relu(F.conv2d(xi, w.bfloat16().float(), b, padding=(kh // 2, kw // 2)))
        yt = yt.permute(0, 2, 3, 1).reshape(P, cout)
        us0 = timeit(lambda: C.conv_fwd([x], wt, g, cout, ref_out[:, :cout], bias=b, act=1, cfg=0))
        line = [f"{name:9s} Cin={cin:3d} N={cout:3d} {kh}x{kw}  auto {us0:6.1f}us ({2 * macs / us0 / 1e6:4.0f}TF)"
                f" err={((ref_out[:, :cout].float() - yt).abs().max().item()):.3f}"]
        for cfg in cfgs:
            out = torch.zeros(P, cp, device=dev, dtype=torch.bfloat16)
            try:
                C.conv_fwd([x], wt, g, cout, out[:, :cout], bias=b, act=1, cfg=cfg)
                torch.cuda.synchronize()
            except RuntimeError as e:  # shape not supported by this variant
                line.append(f"c{cfg} n/a")
                continue
            same = torch.equal(out[:, :cout], ref_out[:, :cout])
            err = (out[:, :cout].float() - yt).abs().max().item()
            us = timeit(lambda: C.conv_fwd([x], wt, g, cout, out[:, :cout], bias=b, act=1, cfg=cfg))
            tag = " ==" if same else f" err={err:.3f}"
            line.append(f"c{cfg} {us:6.1f}us ({2 * macs / us / 1e6:4.0f}TF){tag}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
