#!/usr/bin/env python3
"""Summarise a rocprofv3 --hip-trace CSV: total/max time per HIP API function and the
longest individual calls (host-side stalls: implicit syncs, allocations, blocking copies).
Usage: hip_api_summary.py run_hip_api_trace.csv [--steps N] [--top 25]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    agg = collections.defaultdict(lambda: [0.0, 0, 0.0])
    calls = []
    for r in csv.DictReader(open(args.trace)):
        fn = r.get("Function") or r.get("Operation") or "?"
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        a = agg[fn]
        a[0] += t
        a[1] += 1
        a[2] = max(a[2], t)
        calls.append((t, int(r["Start_Timestamp"]), fn, r.get("Thread_Id", "?")))
    print(f"{'us/step':>10s} {'calls/step':>10s} {'max us':>9s}  function")
    for fn, (t, n, mx) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: args.top]:
        print(f"{t / args.steps:10.1f} {n / args.steps:10.1f} {mx:9.1f}  {fn}")
    print("\nlongest calls:")
    t0 = min(c[1] for c in calls) if calls else 0
    for t, s, fn, tid in sorted(calls, reverse=True)[: args.top]:
        print(f"{t:9.1f} us  at {(s - t0) * 1e-3:12.1f} us  tid {tid}  {fn}")


if __name__ == "__main__":
    main()
