#!/usr/bin/env python3
"""Phases of the last training step in a rocprofv3 SQLite (rocpd) trace, by marker kernels:

  loss           the sequence loss of step k (the boundary kernel) .. its backward
  loop backward  .. lookup_grad_rows (every refinement step's backward; the deferred lookup
                 backward runs once after the last of them)
  tail           .. last kernel before the optimizer (pyramid backward, encoder backward, the
                 batched weight gradients beside it)
  optimizer      clip + AdamW (the native adamw_* kernels, or torch's multi_tensor_apply ones)
  forward        step k+1's forward, up to its loss (encoders, pyramid, 12 refinement steps)

with each phase's wall time, summed kernel time (busy), and the kernels that own most of it;
plus, for the tail, the busy time of the weight-gradient kernels vs the rest.

    python scripts/step_phases.py run_results.db --boundary seq_loss_fwd
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--boundary", default="seq_loss_fwd")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    qcol = "queue_id" if "queue_id" in cols else "stream_id"
    rows = c.execute(f"select name, start, end, stream_id, {qcol} from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.boundary in r[0]]
    if len(idx) < 2:
        raise SystemExit("need two boundary kernels in the trace")
    # one step cycle: this step's loss .. the next step's loss (backward, optimizer, then the
    # next forward); the phases are cut at marker kernels inside it
    step = rows[idx[-2]:idx[-1]]
    t_start = step[0][1]
    names = [r[0] for r in step]
    # the native clip + AdamW op (ops/optim.py) when present, else torch's fused AdamW launches
    if any("adamw_norm_kernel" in n for n in names):
        is_opt = lambda n: "adamw_norm_kernel" in n or "adamw_update_kernel" in n  # noqa: E731
    else:
        is_opt = lambda n: "multi_tensor_apply" in n or "FusedOptimizer" in n  # noqa: E731
    i_bwd = next(i for i, n in enumerate(names) if "seq_loss_bwd" in n)
    i_rows = max((i for i, n in enumerate(names) if "lookup_grad_rows" in n or "lc_gather" in n), default=i_bwd)
    opts = [i for i, n in enumerate(names) if is_opt(n) and i > i_rows]
    i_opt, i_fwd = opts[0], opts[-1] + 1
    phases = [("loss", 0, i_bwd), ("loop backward", i_bwd, i_rows + 1), ("tail", i_rows + 1, i_opt),
              ("optimizer", i_opt, i_fwd), ("forward (next)", i_fwd, len(step))]
    print(f"step wall {(step[-1][2] - t_start) / 1e6:.3f} ms, {len(step)} kernels")
    for name, lo, hi in phases:
        seg = step[lo:hi]
        if not seg:
            continue
        wall = (max(r[2] for r in seg) - seg[0][1]) / 1e6
        agg = defaultdict(float)
        per_stream = defaultdict(float)
        for n, s, e, sid, qid in seg:
            agg[n] += (e - s) / 1e6
            per_stream[(sid, qid)] += (e - s) / 1e6
        busy = sum(agg.values())
        print(f"{name:14s} wall {wall:7.3f} ms  busy {busy:7.3f} ms  kernels {len(seg)}  busy by (stream, queue): "
              + ", ".join(f"{k}: {v:.2f}" for k, v in sorted(per_stream.items())))
        for n, ms in sorted(agg.items(), key=lambda kv: -kv[1])[:a.top]:
            print(f"      {ms:7.3f} ms  {n[:110]}")
        if name in ("tail", "optimizer"):
            wg = sum(ms for n, ms in agg.items() if "wgrad" in n)
            print(f"      -> weight-gradient kernels {wg:.3f} ms busy, other {busy - wg:.3f} ms")
            t0 = seg[0][1]
            for n, s, e, sid, qid in seg:  # when each batched weight gradient ran, on which stream
                if "conv_wgrad" in n or "wgrad_reduce_params" in n:
                    print(f"        {(s - t0) / 1e6:7.3f} .. {(e - t0) / 1e6:7.3f} ms  stream {sid} queue {qid}  {n[:70]}")


if __name__ == "__main__":
    main()
