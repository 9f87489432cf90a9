#!/usr/bin/env python3
"""Run one update-block conv shape repeatedly (for rocprofv3 --pmc counter collection).

    python scripts/conv_one.py zr fwd 6     # shape, pass (fwd|dgrad|wgrad), fwd config
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops import conv as C  # noqa: E402
from scripts.bench_convs import SHAPES  # noqa: E402


def main():
    name, kind = sys.argv[1], sys.argv[2]
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    segs, cout, kh, kw = SHAPES[name]
    B, H, W = 8, 46, 62
    P = B * H * W
    dev = torch.device("cuda")
    cin = sum(r for r, _ in segs)
    cin_p = sum(p for _, p in segs)
    x = torch.randn(P, cin_p, device=dev).bfloat16()
    w = torch.randn(cout, cin, kh, kw, device=dev) * 0.05
    b = torch.randn(cout, device=dev)
    cout_p = (cout + 7) // 8 * 8
    out = torch.empty(P, cout_p, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(P, cout_p, device=dev).bfloat16()
    g = C.geom(B, H, W, kh, kw, kh // 2, kw // 2)
    if kind == "fwd":
        wt = C.pack_fwd(w, segs)
        fn = lambda: C.conv_fwd([x], wt, g, cout, out[:, :cout], bias=b, act=1, cfg=cfg)  # noqa: E731
    elif kind == "dgrad":
        wd = C.pack_dgrad(w, segs)
        dx = torch.empty(P, cin_p, device=dev, dtype=torch.bfloat16)
        gd = C.geom(B, H, W, kh, kw, kh - 1 - kh // 2, kw - 1 - kw // 2)
        fn = lambda: C.conv_fwd([dy], wd, gd, cin_p, dx, epi=C.EPI_GRAD, cfg=cfg)  # noqa: E731
    else:
        wt = C.pack_fwd(w, segs)
        dw = torch.zeros(wt.shape, device=dev)
        db = torch.zeros(cout, device=dev)
        fn = lambda: C.conv_wgrad([x], dy, g, cout, dw, db)  # noqa: E731
    for _ in range(10):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
