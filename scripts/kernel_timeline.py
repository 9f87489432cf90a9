#!/usr/bin/env python3
"""Dispatch-ordered view of the last training step in a rocprofv3 kernel trace: per kernel
its start offset, duration and the idle gap before it (GPU-wide, all streams), plus a summary
of idle time by the kernel that follows the gap (who waits on the host).
Usage: kernel_timeline.py run_kernel_trace.csv --per-step 930 [--list]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--per-step", type=int, required=True, help="kernels per step (the last this many are used)")
    ap.add_argument("--list", action="store_true", help="print every dispatch of the step")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(args.trace)):
        name = r["Kernel_Name"].replace("raft_amd::", "").replace("(anonymous namespace)::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:80],
                     r.get("Grid_Size", r.get("Grid_Size_X", "?"))))
    rows.sort()
    step = rows[-args.per_step:]
    t0 = step[0][0]
    busy_end = t0
    idle = collections.defaultdict(float)
    total_idle = 0.0
    for s, e, name, grid in step:
        gap = max(0, s - busy_end) * 1e-3
        total_idle += gap
        idle[name] += gap
        if args.list:
            print(f"{(s - t0) * 1e-3:9.1f} {(e - s) * 1e-3:8.1f} gap {gap:7.1f}  {grid:>9s}  {name}")
        busy_end = max(busy_end, e)
    span = (busy_end - t0) * 1e-3
    print(f"step span {span:.1f} us, idle {total_idle:.1f} us ({100 * total_idle / span:.1f}%)")
    for name, g in sorted(idle.items(), key=lambda kv: -kv[1])[: args.top]:
        print(f"{g:8.1f} us idle before  {name}")


if __name__ == "__main__":
    main()
