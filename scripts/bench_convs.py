#!/usr/bin/env python3
"""Per-shape timing of the update-block convolutions: HIP implicit-GEMM kernels
(fwd / dgrad / wgrad) vs PyTorch-ROCm (MIOpen) conv2d in bf16 channels-last.

    python scripts/bench_convs.py [--batch 8] [--cfg 0,1,2,3]
Prints one line per (conv, pass) with microseconds and TFLOP/s.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops import conv as C  # noqa: E402

# name: (cin segments, cout, kh, kw)
SHAPES = {
    "convc1": ([(324, 328)], 256, 1, 1),
    "convc2": ([(256, 256)], 192, 3, 3),
    "convf1": ([(2, 8)], 128, 7, 7),
    "convf2": ([(128, 128)], 64, 3, 3),
    "conv": ([(256, 256)], 126, 3, 3),
    "zr": ([(384, 384)], 256, 1, 5),
    "q": ([(384, 384)], 128, 5, 1),
    "zr51": ([(384, 384)], 256, 5, 1),
    "q15": ([(384, 384)], 128, 1, 5),
    "heads": ([(128, 128)], 512, 3, 3),
    "fh2": ([(256, 256)], 2, 3, 3),
    "mask2": ([(256, 256)], 576, 1, 1),
}


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, nargs=2, default=[46, 62])
    ap.add_argument("--cfg", default="")
    ap.add_argument("--iters", type=int, default=12,
                    help="wgrad is timed batched over this many refinement iterations (as in training)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    B, (H, W) = args.batch, args.hw
    P = B * H * W
    cfgs = [int(c) for c in args.cfg.split(",")] if args.cfg else [None]
    tot = {}
    for name, (segs, cout, kh, kw) in SHAPES.items():
        cin = sum(r for r, _ in segs)
        cin_p = sum(p for _, p in segs)
        ph, pw = kh // 2, kw // 2
        macs = P * cout * cin * kh * kw
        x = torch.randn(P, cin_p, device=dev).bfloat16()
        w = torch.randn(cout, cin, kh, kw, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        wt = C.pack_fwd(w, segs)
        wd = C.pack_dgrad(w, segs)
        cout_p = (cout + 7) // 8 * 8
        out = torch.empty(P, max(cout_p, 8), device=dev, dtype=torch.bfloat16)
        dy = torch.randn(P, cout_p, device=dev).bfloat16()
        dx = torch.empty(P, cin_p, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(wt.shape, device=dev)
        db = torch.zeros(cout, device=dev)
        T = args.iters
        xT = torch.randn(T * P, cin_p, device=dev).bfloat16()
        dyT = torch.randn(T * P, cout_p, device=dev).bfloat16()
        gT = C.geom(T * B, H, W, kh, kw, ph, pw)
        g = C.geom(B, H, W, kh, kw, ph, pw)
        gd = C.geom(B, H, W, kh, kw, kh - 1 - ph, kw - 1 - pw)
        line = [f"{name:7s} M={P} N={cout:4d} K={cin * kh * kw:5d}"]
        for cfg in cfgs:
            c = cfg or 0
            tf = timeit(lambda: C.conv_fwd([x], wt, g, cout, out[:, :cout], bias=b, act=1, cfg=c))
            td = timeit(lambda: C.conv_fwd([dy], wd, gd, cin_p, dx, epi=C.EPI_GRAD, cfg=c))
            line.append(f"cfg{cfg}: fwd {tf:7.1f}us ({2 * macs / tf / 1e6:5.0f}TF) dgrad {td:7.1f}us "
                        f"({2 * macs / td / 1e6:5.0f}TF)")
        tw = timeit(lambda: C.conv_wgrad([xT], dyT, gT, cout, dw, db, False), reps=5) / T
        tw0 = timeit(lambda: C.conv_wgrad([xT], dyT, gT, cout, dw, None, False), reps=5) / T
        line.append(f"wgrad/iter (x{T} batched) {tw:7.1f}us (no db {tw0:6.1f}us {2 * macs / tw0 / 1e6:5.0f}TF)")
        # MIOpen reference
        xt = x[:, :cin].float().reshape(B, H, W, cin).permute(0, 3, 1, 2).bfloat16().contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        wtt = w.bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
        bt = b.bfloat16().requires_grad_(True)
        tmf = timeit(lambda: F.conv2d(xt, wtt, bt, padding=(ph, pw)))
        yt = F.conv2d(xt, wtt, bt, padding=(ph, pw))
        gy = torch.randn_like(yt)
        tmb = timeit(lambda: torch.autograd.grad(yt, (xt, wtt, bt), gy, retain_graph=True))
        line.append(f"| miopen fwd {tmf:7.1f}us bwd(d+w) {tmb:7.1f}us")
        # same-FLOP plain GEMM through hipBLASLt (torch.mm): what a tuned library reaches at this M,N,K
        am = torch.randn(P, cin * kh * kw, device=dev).bfloat16()
        bm = torch.randn(cin * kh * kw, cout, device=dev).bfloat16()
        tg = timeit(lambda: torch.mm(am, bm))
        line.append(f"| blas gemm {tg:7.1f}us ({2 * macs / tg / 1e6:5.0f}TF)")
        print("  ".join(line), flush=True)
        tot.setdefault("ours_fwd", 0.0)
        tot["ours_fwd"] = tot["ours_fwd"] + tf
        tot["ours_bwd"] = tot.get("ours_bwd", 0.0) + td + tw
        tot["miopen_fwd"] = tot.get("miopen_fwd", 0.0) + tmf
        tot["miopen_bwd"] = tot.get("miopen_bwd", 0.0) + tmb
    print({k: round(v, 1) for k, v in tot.items()}, "us per iteration (one of each conv)")


if __name__ == "__main__":
    main()
