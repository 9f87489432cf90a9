#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite (rocpd) database: the last ``--steps`` steps
(split at each launch of ``--boundary``), total ms per step, calls per step, mean us.

    python scripts/rocpd_summary.py gpurun_out/measure/prof_fp32/run_results.db \
        --boundary convex_up_fwd --steps 3 --top 40
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--boundary", default=None, help="substring of a kernel launched once per step")
    ap.add_argument("--steps", type=int, default=3, help="summarise the last N steps")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default=None)
    ap.add_argument("--by-grid", action="store_true", help="split each kernel by its launch grid (shapes)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    if a.by_grid:
        cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
        gx = next((x for x in ("grid_size_x", "grid_x", "grid_size") if x in cols), None)
        gy = next((x for x in ("grid_size_y", "grid_y") if x in cols), None)
        sel = (f"'grid=' || {gx}" + (f" || 'x' || {gy}" if gy else "") + " || ' ' || name") if gx else "name"
        rows = c.execute(f"select {sel}, start, end from kernels order by start").fetchall()
    else:
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if a.boundary:
        idx = [i for i, r in enumerate(rows) if a.boundary in r[0]]
        if len(idx) > a.steps:
            rows = rows[idx[-a.steps - 1] + 1: idx[-1] + 1]
            n = a.steps
        else:
            n = 1
    else:
        n = 1
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in rows:
        agg[name][0] += 1
        agg[name][1] += (e - s) / 1e6
    busy = sum(v[1] for v in agg.values()) / n
    wall = (rows[-1][2] - rows[0][1]) / 1e6 / n if rows else 0.0
    lines = [f"steps={n} kernels/step={len(rows) / n:.0f} busy/step={busy:.3f}ms wall/step={wall:.3f}ms"]
    for name, (cnt, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        lines.append(f"{ms / n:9.3f} ms/step {100 * ms / n / max(busy, 1e-9):5.1f}%  calls/step={cnt / n:6.1f}  "
                     f"{1000 * ms / cnt:8.1f} us/call  {name[:150]}")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
