#!/usr/bin/env python3
"""Per-op timing of the native encoder kernels on the bench shapes (RAFT-base feature
encoder, 2 x batch images at 368x496): forward, data gradient and weight gradient of
every conv, with achieved TFLOP/s (useful MACs only).

    python scripts/bench_enc.py [--images 16] [--size 368 496]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=16)
    ap.add_argument("--size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from raft_ros_amd.ops._ext import ops
    o = ops()
    dev = torch.device("cuda", 0)
    B = args.images
    H, W = args.size[0] // 2, args.size[1] // 2
    # (name, Cin, Cout, k, stride, pad, input H, input W)
    convs = [("stem7x7s2", 8, 64, 7, 2, 3, 2 * H, 2 * W),
             ("l1_3x3", 64, 64, 3, 1, 1, H, W),
             ("l2_3x3s2", 64, 96, 3, 2, 1, H, W),
             ("l2_1x1s2", 64, 96, 1, 2, 0, H, W),
             ("l2_3x3", 96, 96, 3, 1, 1, H // 2, W // 2),
             ("l3_3x3s2", 96, 128, 3, 2, 1, H // 2, W // 2),
             ("l3_1x1s2", 96, 128, 1, 2, 0, H // 2, W // 2),
             ("l3_3x3", 128, 128, 3, 1, 1, H // 4, W // 4),
             ("out_1x1", 128, 256, 1, 1, 0, H // 4, W // 4)]

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    print(f"{'conv':12s} {'fwd us':>8s} {'TF/s':>6s} {'dgrad us':>9s} {'TF/s':>6s} {'wgrad us':>9s} {'TF/s':>6s}")
    for name, ci, co, k, s, p, hi, wi in convs:
        x = torch.randn(B, hi, wi, ci, device=dev).bfloat16()
        w = torch.randn(co, ci if ci != 8 else 3, k, k, device=dev).contiguous(memory_format=torch.channels_last)
        b = torch.randn(co, device=dev)
        y, _ = o.enc_conv_fwd(x, w, b, s, p, True)
        ho, wo = y.shape[1], y.shape[2]
        macs = B * ho * wo * co * (w.shape[1] * k * k)
        tf = lambda us: 2 * macs / (us * 1e-6) / 1e12  # noqa: E731
        t_f = timeit(lambda: o.enc_conv_fwd(x, w, b, s, p, True)) * 1e3
        dy = torch.randn_like(y)
        if ci % 8 == 0 and name != "stem7x7s2":
            t_d = timeit(lambda: o.enc_conv_dgrad([dy], [w], [s], [p], hi, wi, None, None)) * 1e3
        else:
            t_d = float("nan")
        dw = torch.empty_like(w)
        db = torch.empty(co, device=dev)
        t_w = timeit(lambda: o.enc_conv_wgrad(x, dy, dw, db, s, p, False, False)) * 1e3
        print(f"{name:12s} {t_f:8.1f} {tf(t_f):6.0f} {t_d:9.1f} {tf(t_d):6.0f} {t_w:9.1f} {tf(t_w):6.0f}", flush=True)


if __name__ == "__main__":
    main()
