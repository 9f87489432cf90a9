#!/usr/bin/env python3
"""Correlation-volume GEMM timing (the dense pyramid build, ops/corr.py _BuildPyramid):
v2 store-oriented kernel vs the generic one (cfg=1), at the training and 1080p shapes; and
the radius-4 lookup forward (bf16 volume -> padded bf16 features), the per-lookup backward
(bf16 window gradient -> read-modify-write of fp32 level gradients) and the deferred
backward of a 12-lookup step (all window gradients -> bf16 level-gradient rows, one pass).

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


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1000


def levels_of(buf, H, W, levels=4):
    out, off = [], 0
    for l in range(levels):
        Hl, Wl = H >> l, W >> l
        nb = -(-Wl // 16)
        out.append(buf.as_strided((buf.shape[0], nb, Hl, 16), (buf.shape[1], Hl * 16, 16, 1), off))
        off += nb * 16 * Hl
    return out


def main():
    dev = torch.device("cuda")
    k = ops()
    for name, B, H, W in (("train 8x368x496", 8, 46, 62), ("sintel 1x440x1024", 1, 55, 128), ("1080p", 1, 135, 240)):
        HW, ld, C = H * W, ld_of(H, W), 256
        A = torch.randn(B, HW, C, device=dev).bfloat16()
        Bm = torch.randn(B, ld, C, device=dev).bfloat16()
        out = torch.empty(B * HW, ld, device=dev, dtype=torch.bfloat16)
        line = [f"{name:18s} M={HW} N={ld} K={C} batch={B}"]
        for cfg in (0, 11, 12, 8, 0, 11, 12, 1):
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
            if cfg == 0:
                ref0 = out.clone()
            elif cfg >= 2:  # same tiles in another order (2-5: bitwise equal; v3 6-8: operands swapped)
                line.append("==" if torch.equal(out, ref0) else
                            f"maxdiff {(out.float() - ref0.float()).abs().max().item():.1e}")
        print("  ".join(line), flush=True)
        # lookups on this volume (the flow-sized random walk of a mid-training iteration)
        lv = levels_of(out, H, W)
        ys, xs = torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev), indexing="ij")
        coords = torch.stack([xs, ys]).float()[None].repeat(B, 1, 1, 1)
        coords = (coords + 8 * torch.randn_like(coords)).contiguous()
        feat = torch.empty(B, H, W, 328, device=dev, dtype=torch.bfloat16)
        fwd = timed(lambda: k.corr_lookup_into(lv, coords, 4, feat, None, None))
        dbuf = torch.zeros(B * HW, ld, device=dev)
        dlv = levels_of(dbuf, H, W)
        g = torch.randn(B, H, W, 328, device=dev).bfloat16()
        bwd = timed(lambda: k.corr_lookup_backward_(dlv, coords, g, 4))
        rows = torch.empty(B * HW, ld, device=dev, dtype=torch.bfloat16)
        segs, o = [], 0
        for l in range(4):
            segs += [o, H >> l, W >> l]
            o += -(-(W >> l) // 16) * 16 * (H >> l)
        cs, gs = [coords] * 12, [g] * 12
        rows_us = {}  # rows longer than the kernel's LDS budget keep the per-lookup pass
        if ld <= 15616:
            for T in (1, 4, 12):
                rows_us[T] = timed(lambda: k.corr_lookup_grad_rows(rows, cs[:T], gs[:T], segs, 4, False), n=5)
        dfr = "  ".join(f"T={T}: {v:6.1f} us" for T, v in rows_us.items())
        print(f"{'':18s} lookup fwd {fwd:7.1f} us  bwd per lookup {bwd:7.1f} us (x12 = {12 * bwd:7.1f})  "
              f"deferred bwd of T lookups {dfr}  ({B * HW} queries)", flush=True)


if __name__ == "__main__":
    main()
