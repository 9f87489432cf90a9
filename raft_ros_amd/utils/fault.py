"""Fault injection for failure-detection tests ("a fault-injection hook
in tests (kill a rank -> job aborts cleanly)").  The reference has no failure handling at
all (train.py:136-214 runs until an exception or a hang).

``RAFT_FAULT_INJECT`` selects one fault, e.g. ``"rank=1,step=2,kind=exit"``:

* ``kind=exit``  -- the rank dies without any cleanup (``os._exit(code)``), like a crashed or
  OOM-killed process; the other ranks must not hang (the launcher tears the job down, a
  collective timeout backs that up);
* ``kind=raise`` -- the rank raises ``InjectedFault`` from the training loop;
* ``kind=nan``   -- the rank's loss becomes NaN for that step, which exercises the
  non-finite-gradient guard (the step must be skipped on every rank, weights unchanged);
* ``kind=hang``  -- the rank sleeps ``secs`` seconds (default 3600) before the step, which
  exercises the collective timeout of the process group.

``rank`` defaults to every rank, ``step`` to 0.  With the variable unset every hook is a
no-op costing one attribute check.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Optional

import torch

ENV = "RAFT_FAULT_INJECT"
KINDS = ("exit", "raise", "nan", "hang")


class InjectedFault(RuntimeError):
    pass


@dataclass(frozen=True)
class Fault:
    kind: str
    step: int = 0
    rank: Optional[int] = None
    code: int = 17
    secs: float = 3600.0

    def hits(self, step: int, rank: int) -> bool:
        return step == self.step and (self.rank is None or self.rank == rank)


def parse(spec: str) -> Fault:
    fields = {}
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        key, sep, val = part.partition("=")
        if not sep:
            raise ValueError(f"{ENV}: expected key=value, got {part!r}")
        fields[key.strip()] = val.strip()
    kind = fields.pop("kind", None)
    if kind not in KINDS:
        raise ValueError(f"{ENV}: kind must be one of {KINDS}, got {kind!r}")
    out = Fault(kind=kind,
                step=int(fields.pop("step", 0)),
                rank=int(fields["rank"]) if "rank" in fields else None,
                code=int(fields.pop("code", 17)),
                secs=float(fields.pop("secs", 3600.0)))
    fields.pop("rank", None)
    if fields:
        raise ValueError(f"{ENV}: unknown keys {sorted(fields)}")
    return out


def from_env() -> Optional[Fault]:
    spec = os.environ.get(ENV, "")
    return parse(spec) if spec else None


class Injector:
    """Per-run hook object; ``before_step`` runs before the forward pass, ``on_loss`` may
    replace the loss."""

    def __init__(self, fault: Optional[Fault], rank: int):
        self.fault = fault
        self.rank = rank

    @classmethod
    def from_env(cls, rank: int) -> "Injector":
        return cls(from_env(), rank)

    def before_step(self, step: int) -> None:
        f = self.fault
        if f is None or not f.hits(step, self.rank):
            return
        if f.kind == "exit":
            print(f"[fault] rank {self.rank}: exiting with code {f.code} at step {step}", flush=True)
            os._exit(f.code)
        if f.kind == "raise":
            raise InjectedFault(f"injected fault on rank {self.rank} at step {step}")
        if f.kind == "hang":
            print(f"[fault] rank {self.rank}: hanging {f.secs:.0f}s at step {step}", flush=True)
            time.sleep(f.secs)

    def on_loss(self, step: int, loss: torch.Tensor) -> torch.Tensor:
        f = self.fault
        if f is None or f.kind != "nan" or not f.hits(step, self.rank):
            return loss
        return loss * float("nan")
