"""Training logger (reference train.py:89-133).

Keeps the reference's console format -- every ``SUM_FREQ`` steps
``[  step,  lr] m1, m2, ...`` with metrics averaged over the window and sorted
by name -- and adds a JSONL log (one record per print and per validation) and
pairs/s throughput.  TensorBoard is used when ``torch.utils.tensorboard`` is
importable (it is optional; the package is not installed in this image).
Only rank 0 writes, but with several ranks the window averages are all-reduced
first (``reduce_fn``, a collective every rank enters at the same step), so the
printed metrics are over the whole global batch, not rank 0's shard.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

SUM_FREQ = 100


class Logger:
    def __init__(self, model=None, scheduler=None, log_dir: str = "runs", enabled: bool = True,
                 sum_freq: int = SUM_FREQ, pairs_per_step: int = 0, reduce_fn=None):
        self.model = model
        self.scheduler = scheduler
        self.total_steps = 0
        self.running_loss: Dict[str, float] = {}
        self.enabled = enabled
        self.sum_freq = sum_freq
        self.pairs_per_step = pairs_per_step
        self.reduce_fn = reduce_fn  # {name: value} -> {name: mean over ranks}; called on every rank
        self.writer = None
        self.log_dir = log_dir
        self.jsonl = None
        self._t = time.perf_counter()
        if enabled:
            os.makedirs(log_dir, exist_ok=True)
            self.jsonl = open(os.path.join(log_dir, "metrics.jsonl"), "a")

    def _tb(self):
        if self.writer is None and self.enabled:
            try:
                from torch.utils.tensorboard import SummaryWriter

                self.writer = SummaryWriter(self.log_dir)
            except Exception:  # tensorboard not installed
                self.writer = False
        return self.writer or None

    def _lr(self) -> float:
        # float(): a capturable optimizer (train.py --graph) keeps lr in a device tensor
        return float(self.scheduler.get_last_lr()[0]) if self.scheduler is not None else 0.0

    def _print_training_status(self):
        keys = sorted(self.running_loss)
        means = {k: float(self.running_loss[k]) / self.sum_freq for k in keys}
        if self.reduce_fn is not None:
            means = self.reduce_fn(means)
        vals = [means[k] for k in keys]
        now = time.perf_counter()
        rate = self.pairs_per_step * self.sum_freq / max(now - self._t, 1e-9) if self.pairs_per_step else 0.0
        self._t = now
        if self.enabled:
            head = "[{:6d}, {:10.7f}] ".format(self.total_steps + 1, self._lr())
            print(head + ("{:10.4f}, " * len(vals)).format(*vals), flush=True)
            rec = {"step": self.total_steps + 1, "lr": self._lr(), **dict(zip(keys, vals))}
            if rate:
                rec["pairs_per_s"] = rate
            self.jsonl.write(json.dumps(rec) + "\n")
            self.jsonl.flush()
            w = self._tb()
            if w:
                for k, v in zip(keys, vals):
                    w.add_scalar(k, v, self.total_steps)
        self.running_loss = {}

    def push(self, metrics: Dict[str, float]):
        """Accumulate a step's metrics; device tensors stay on the device (no host sync)
        until the window is printed."""
        self.total_steps += 1
        for k, v in metrics.items():
            v = v.detach() if hasattr(v, "detach") else float(v)
            self.running_loss[k] = self.running_loss.get(k, 0.0) + v
        if self.total_steps % self.sum_freq == self.sum_freq - 1:
            self._print_training_status()

    def write_dict(self, results: Dict[str, float]):
        if not self.enabled:
            return
        self.jsonl.write(json.dumps({"step": self.total_steps, "validation": {k: float(v) for k, v in results.items()}}) + "\n")
        self.jsonl.flush()
        w = self._tb()
        if w:
            for k, v in results.items():
                w.add_scalar(k, v, self.total_steps)

    def close(self):
        if self.writer:
            self.writer.close()
        if self.jsonl:
            self.jsonl.close()
