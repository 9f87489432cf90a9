#!/usr/bin/env python3
"""1x1 weight gradients of the refinement step (batched over 12 iterations, config #2):
the hand-written conv_wgrad (wgrad v2, fused bias) vs hipBLASLt through torch.mm(dY^T, X,
out_dtype=fp32) (+ the bias column sum), same operands.

    python scripts/bench_wgrad_blas.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops import conv as C  # noqa: E402

SHAPES = {"convc1": (328, 256), "mask2": (256, 576), "convf1(7x7 as K=392)": None}


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0


def main():
    dev = torch.device("cuda")
    B, H, W, T = 8, 46, 62, 12
    P = T * B * H * W
    for name, (cin, cout) in ((k, v) for k, v in SHAPES.items() if v is not None):
        x = torch.randn(P, cin, device=dev).bfloat16()
        dy = torch.randn(P, cout, device=dev).bfloat16()
        g = C.geom(T * B, H, W, 1, 1, 0, 0)
        dw = torch.zeros(cout, C._round(cin, 64), device=dev)
        db = torch.zeros(cout, device=dev)
        t_ours = timeit(lambda: C.conv_wgrad([x], dy, g, cout, dw, db, False))
        t_blas = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        t_bsum = timeit(lambda: dy.sum(0, dtype=torch.float32))
        ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
        C.conv_wgrad([x], dy, g, cout, dw, db, False)
        err = float((dw[:, :cin] - ref).norm() / ref.norm())
        gb = (P * (cin + cout) * 2) / 1e9
        print(f"{name:8s} P={P} N={cout} K={cin}: conv_wgrad {t_ours:7.1f} us (with bias) | torch.mm fp32-out "
              f"{t_blas:7.1f} us + bias sum {t_bsum:6.1f} us | operand bytes {gb:.2f} GB -> floor "
              f"{gb / 5.5e3 * 1e6:.0f} us at 5.5 TB/s | rel diff {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
