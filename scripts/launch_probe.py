#!/usr/bin/env python3
"""Host cost per runtime operation on this box (csrc/bindings.cpp launch_probe): kernel launches
with a small / ConvFwdArgs-sized argument block, a cross-stream event fork, a 1 MB allocation,
and the Python -> torch.ops dispatch of a native op (one launch inside) -- the pieces the eager
training step's ~15 ms of host issue is made of.

    python scripts/launch_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops._ext import ops  # noqa: E402


def main():
    k = ops()
    torch.cuda.init()
    side = torch.cuda.Stream()
    n = 2000
    for _ in range(2):  # warm-up, then report
        rows = {
            "launch, 8-byte args (us)": k.launch_probe(n, 0),
            "launch, ConvFwdArgs args (us)": k.launch_probe(n, 1),
            "event record + wait on another stream (us)": k.launch_probe(n, 2, side.cuda_stream),
            "at::empty 1 MB (us)": k.launch_probe(n, 3),
        }
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            k.launch_probe(1, 0)
        rows["python -> torch.ops call of a 1-launch op (us)"] = (time.perf_counter() - t0) / n * 1e6
        x = torch.zeros(1, 2, 4, 4, device="cuda")
        y, f = torch.empty_like(x), torch.empty_like(x)
        d = torch.zeros(16, 8, device="cuda")
        t0 = time.perf_counter()
        for _ in range(n):
            k.apply_delta(x, d, y, f)
        rows["python -> apply_delta (4 tensor args, 1 launch) (us)"] = (time.perf_counter() - t0) / n * 1e6
        t0 = time.perf_counter()
        for _ in range(n):
            side.wait_stream(torch.cuda.current_stream())
        rows["torch Stream.wait_stream (us)"] = (time.perf_counter() - t0) / n * 1e6
        torch.cuda.synchronize()
    for name, v in rows.items():
        print(f"{name:55s} {v:8.2f}")


if __name__ == "__main__":
    main()
