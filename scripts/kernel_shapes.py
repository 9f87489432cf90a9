#!/usr/bin/env python3
"""Group a rocprofv3 kernel trace by (kernel, grid size): which launch shapes of a kernel
cost the time.  Usage: kernel_shapes.py run_kernel_trace.csv [--top 30] [--steps N]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this (per-step numbers)")
    args = ap.parse_args()
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(args.trace)):
        key = (r["Kernel_Name"].replace("raft_amd::", "").replace("(anonymous namespace)::", "")[:70],
               r.get("Grid_Size", r.get("Grid_Size_X", "?")), r.get("LDS_Block_Size", r.get("Lds_Size", "?")))
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        agg[key][0] += t
        agg[key][1] += 1
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
    print(f"{'ms/step':>8s} {'calls':>6s} {'us/call':>8s}  grid      lds    kernel")
    for (name, grid, lds), (t, n) in rows[: args.top]:
        print(f"{t / args.steps:8.3f} {n / args.steps:6.1f} {1e3 * t / n:8.1f}  {grid:>9s} {lds:>6s}  {name}")


if __name__ == "__main__":
    main()
