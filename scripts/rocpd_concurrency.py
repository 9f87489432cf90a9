#!/usr/bin/env python3
"""Concurrency profile of a multi-stream step from a rocprofv3 SQLite database: over the last
``--steps`` steps (split at ``--boundary``), the wall time with 0 / 1 / 2 / 3+ kernels in
flight, and -- for the time with exactly one kernel running (the serial critical path) --
which kernels own it.

    python scripts/rocpd_concurrency.py gpurun_out/measure/prof_train/run_results.db --boundary seq_loss_fwd
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--boundary", default="seq_loss_fwd")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--gaps", type=int, default=40, help="list the N longest idle gaps of the last step")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.boundary in r[0]]
    rows = rows[idx[-a.steps - 1] + 1: idx[-1] + 1]
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    ev = []
    for i, (n, s, e, st) in enumerate(rows):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    hist = defaultdict(float)
    solo = defaultdict(float)
    idle_before = defaultdict(float)  # zero-in-flight gaps, by the kernel that ends them
    ngaps = 0
    gaps = []  # (duration, time, previous kernel to end, next kernel)
    last_end = None
    last = t0
    for t, d, i in ev:
        if t > last:
            k = len(active)
            hist[min(k, 3)] += t - last
            if k == 1:
                solo[rows[next(iter(active))][0]] += t - last
            if k == 0 and d > 0:
                idle_before[rows[i][0]] += t - last
                ngaps += 1
                gaps.append((t - last, t, rows[last_end][0] if last_end is not None else "-", rows[i][0], i))
        if d < 0:
            last_end = i
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    wall = (t1 - t0) / a.steps / 1e6
    print(f"wall/step {wall:.3f} ms; streams {sorted({r[3] for r in rows})}")
    for k in range(4):
        print(f"  {k}{'+' if k == 3 else ' '} kernels in flight: {hist[k] / a.steps / 1e6:7.3f} ms/step "
              f"({100 * hist[k] / (t1 - t0):5.1f} %)")
    print(f"zero-in-flight gaps: {ngaps / a.steps:.0f}/step, mean {hist[0] / max(ngaps, 1) / 1e3:.2f} us; "
          "idle time by the kernel that ends the gap:")
    for n, v in sorted(idle_before.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"  {v / a.steps / 1e6:7.3f} ms/step  {n[:140]}")
    if a.gaps:
        t_last = sorted(r[1] for r in rows)[-(len(rows) // a.steps)]  # ~start of the last step
        print(f"longest idle gaps of the last step (us, kernel index in step, previous -> next):")
        per = len(rows) // a.steps
        for g, t, prev, nxt, i in sorted([x for x in gaps if x[1] >= t_last], reverse=True)[:a.gaps]:
            print(f"  {g / 1e3:7.1f}  #{i % per:4d}  {prev[:60]:60s} -> {nxt[:70]}")
    print("serial (exactly one kernel in flight) time by kernel:")
    for n, v in sorted(solo.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"  {v / a.steps / 1e6:7.3f} ms/step  {n[:140]}")


if __name__ == "__main__":
    main()
