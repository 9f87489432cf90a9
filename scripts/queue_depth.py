#!/usr/bin/env python3
"""How far can the host run ahead of the GPU on one HIP stream?  Issue a long run of ~20 us
spin kernels and time each launch on the host: while the stream's queue has room a launch
returns in a few microseconds; once it is full the host blocks for about one kernel's GPU
time per launch.  The index of the first blocking launch is the in-flight depth.

    python scripts/queue_depth.py [--n 3000] [--cycles 50000]
"""
from __future__ import annotations

import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3000)
    ap.add_argument("--cycles", type=int, default=50000)
    args = ap.parse_args()
    torch.cuda.init()
    for _ in range(10):
        torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(args.cycles)
    e.record()
    torch.cuda.synchronize()
    k_us = 1e3 * s.elapsed_time(e)
    for label, stream in (("default stream", torch.cuda.current_stream()), ("new stream", torch.cuda.Stream())):
        with torch.cuda.stream(stream):
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.n):
                t0 = time.perf_counter()
                torch.cuda._sleep(args.cycles)
                ts.append(1e6 * (time.perf_counter() - t0))
            torch.cuda.synchronize()
        slow = [i for i, t in enumerate(ts) if t > 0.5 * k_us]
        first = slow[0] if slow else None
        tail = ts[first:] if first is not None else []
        print(f"{label}: kernel {k_us:.1f} us on the GPU; host launch {sum(ts[:100]) / 100:.1f} us while the queue "
              f"has room; first blocking launch at #{first}; after it mean {sum(tail) / max(len(tail), 1):.1f} us "
              f"({len(slow)} of {args.n} launches blocked)", flush=True)


if __name__ == "__main__":
    main()
