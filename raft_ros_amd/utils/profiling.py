"""Tracing hooks: ROCTX ranges around the phases of a step and an optional
torch.profiler capture (``RAFT_PROFILE=<dir>`` or ``--profile_dir``).

rocprofv3 picks the ROCTX ranges up with ``--marker-trace``; the kernel-level
numbers committed under ``profiles/`` come from ``rocprofv3 --kernel-trace
--stats`` (see scripts/gpu_check.sh and scripts/kernel_summary.py).
"""
from __future__ import annotations

import contextlib
import os

import torch


@contextlib.contextmanager
def trace_range(name: str):
    """A named ROCTX range (no-op on CPU)."""
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)  # ROCTX on ROCm builds
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


def maybe_profiler(out_dir: str | None = None, wait: int = 2, warmup: int = 2, active: int = 3):
    """torch.profiler schedule writing a chrome trace + a kernel table into ``out_dir``."""
    out_dir = out_dir or os.environ.get("RAFT_PROFILE")
    if not out_dir:
        return contextlib.nullcontext(None)
    os.makedirs(out_dir, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)

    def on_ready(prof):
        prof.export_chrome_trace(os.path.join(out_dir, f"trace_{prof.step_num}.json"))
        with open(os.path.join(out_dir, "kernels.txt"), "w") as f:
            sort = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
            f.write(prof.key_averages().table(sort_by=sort, row_limit=60))

    return torch.profiler.profile(activities=acts, schedule=torch.profiler.schedule(wait=wait, warmup=warmup,
                                                                                      active=active),
                                  on_trace_ready=on_ready)
