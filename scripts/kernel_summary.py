#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace over the steady-state steps only.

MIOpen's first-call tuning (cudnn.benchmark) launches thousands of naive
candidate kernels during warmup, which swamps ``--stats``.  This script reads
``*_kernel_trace.csv``, splits it into training steps at every occurrence of a
boundary kernel (one launch per step), drops the first ``--skip`` steps and
prints / writes a per-step breakdown grouped by kernel name.

    python scripts/kernel_summary.py gpurun_out/prof/run_kernel_trace.csv \
        --boundary seq_loss_fwd --skip 2 --out profiles/x.csv
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\s+", " ", name)
    return name[:140]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--boundary", default="seq_loss_fwd")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--every", type=int, default=1, help="boundary launches per step")
    ap.add_argument("--out", default=None)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cuts = [i for i, r in enumerate(rows) if re.search(args.boundary, r["Kernel_Name"])]
    cuts = cuts[args.every - 1::args.every]
    if len(cuts) <= args.skip:
        raise SystemExit(f"only {len(cuts)} boundary kernels found")
    lo, hi = cuts[args.skip - 1] + 1 if args.skip > 0 else 0, cuts[-1] + 1
    steps = len(cuts) - args.skip
    sel = rows[lo:hi]
    agg = defaultdict(lambda: [0, 0.0])
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += d
    busy = sum(v[1] for v in agg.values())
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6
    print(f"steps={steps} kernels/step={len(sel) / steps:.0f} busy/step={busy / steps:.2f}ms "
          f"wall/step={wall / steps:.2f}ms")
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for name, (n, t) in items[: args.top]:
        print(f"{t / steps:8.3f} ms/step {100 * t / busy:5.1f}%  calls/step={n / steps:6.1f}  {name}")
    if args.out:
        with open(args.out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "ms_per_step", "pct_busy", "calls_per_step"])
            for name, (n, t) in items:
                w.writerow([name, f"{t / steps:.4f}", f"{100 * t / busy:.2f}", f"{n / steps:.1f}"])
            w.writerow(["__total_busy__", f"{busy / steps:.4f}", "100", f"{len(sel) / steps:.0f}"])
            w.writerow(["__wall__", f"{wall / steps:.4f}", "", ""])


if __name__ == "__main__":
    main()
