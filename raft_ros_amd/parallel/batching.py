"""Global-batch semantics under one process per GPU (reference ``train.py:138,172-175``).

The reference's ``--batch_size`` is the GLOBAL batch: ``nn.DataParallel`` scatters every
batch of B samples over its replicas and reduces the replicas' gradients into one, so the
update is the gradient of the mean loss over all B samples, whatever the GPU count.  The
standard schedule (``train_standard.sh:3-6``) uses B = 10 (chairs) and B = 6 (things /
sintel / kitti), which do not divide 4 or 8 ranks.  This module keeps that semantics exactly:

* :func:`rank_batch_sizes` splits B over the ranks.  ``"balanced"`` (default) gives the
  first ``B % W`` ranks one extra sample (10 over 8 -> 2,2,1,1,1,1,1,1); ``"chunk"``
  reproduces DataParallel's own scatter, ``torch.chunk`` (10 over 8 -> 2,2,2,2,2,0,0,0), so
  per-replica BatchNorm statistics are grouped exactly like the reference's replicas.  With
  B < W some ranks get no sample in either policy (6 over 8 -> six ranks of 1, two idle).
* :class:`GlobalBatchSampler` draws the SAME shuffled global batch on every rank (one
  permutation per epoch from ``seed + epoch``) and hands rank r its slice, so every rank runs
  ``len(dataset) // B`` steps per epoch and the ranks' samples are disjoint -- the reference's
  ``DataLoader(shuffle=True, drop_last=True)`` batches, split like DataParallel splits them.
* :func:`loss_weight` = ``b_r * W / B``.  Each rank's loss is a mean over its own b_r
  samples; scaled by this weight, the AVG all-reduce of the gradients (GradSync or DDP)
  yields ``sum_r (b_r / B) grad(loss_r)`` = the gradient of the mean loss over the B samples.
  Logged metrics are weighted the same way.  An idle rank (b_r = 0) runs no forward under
  GradSync and contributes zeros to the all-reduce.

BatchNorm (only the base context encoder in the chairs stage has trainable statistics;
every later stage freezes BN, ``train.py:147-148``): per-rank statistics by default, as in
the reference's DataParallel replicas -- a 1-image rank normalises over that image's H x W
pixels, which is well defined.  ``--sync_bn`` instead normalises over the whole global
batch; it needs equal per-rank batches (the native encoder all-gathers fixed-shape
per-tile statistics), which :func:`check_sync_bn` enforces with a clear error.
"""
from __future__ import annotations

from typing import Iterator, List, Sequence

import torch
from torch.utils.data import Sampler

POLICIES = ("balanced", "chunk")


def rank_batch_sizes(global_batch: int, world: int, policy: str = "balanced") -> List[int]:
    """Per-rank sample counts summing to ``global_batch`` (see the module docstring)."""
    if global_batch < 1 or world < 1:
        raise ValueError(f"global batch {global_batch} / world size {world} must be >= 1")
    if policy == "balanced":
        base, rem = divmod(global_batch, world)
        return [base + (1 if r < rem else 0) for r in range(world)]
    if policy == "chunk":  # torch.chunk(B, world): DataParallel's scatter (torch/nn/parallel/comm.py)
        step = -(-global_batch // world)
        return [max(0, min(step, global_batch - r * step)) for r in range(world)]
    raise ValueError(f"batch split policy {policy!r}: one of {POLICIES}")


def rank_offset(sizes: Sequence[int], rank: int) -> int:
    return int(sum(sizes[:rank]))


def loss_weight(sizes: Sequence[int], rank: int) -> float:
    """Scale of rank ``rank``'s mean loss so that averaging gradients over the ranks gives the
    full-batch gradient: ``b_r * W / B``."""
    total = sum(sizes)
    return sizes[rank] * len(sizes) / total


def check_sync_bn(sizes: Sequence[int]) -> None:
    if len(set(sizes)) != 1:
        raise ValueError(f"--sync_bn needs equal per-rank batches; the global batch splits as {list(sizes)} -- "
                         "use a batch size divisible by the GPU count, or per-rank BatchNorm (the default)")


class GlobalBatchSampler(Sampler[List[int]]):
    """Batch sampler: every rank draws the same shuffled global batches of ``sum(sizes)``
    indices and yields its own slice of each (``drop_last`` semantics: a final partial global
    batch is dropped, as the reference's DataLoader does)."""

    def __init__(self, n: int, sizes: Sequence[int], rank: int, seed: int = 0, shuffle: bool = True):
        self.n = int(n)
        self.sizes = [int(s) for s in sizes]
        self.rank = int(rank)
        self.global_batch = sum(self.sizes)
        self.lo = rank_offset(self.sizes, rank)
        self.hi = self.lo + self.sizes[rank]
        self.seed = int(seed)
        self.shuffle = shuffle
        self.epoch = 0
        if self.n < self.global_batch:
            raise ValueError(f"dataset of {n} samples is smaller than the global batch {self.global_batch}")

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __len__(self) -> int:
        return self.n // self.global_batch

    def __iter__(self) -> Iterator[List[int]]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g)
        else:
            order = torch.arange(self.n)
        B = self.global_batch
        for i in range(len(self)):
            yield order[i * B + self.lo:i * B + self.hi].tolist()


class IdleLoader:
    """Loader of a rank with no sample in the global batch: yields ``None`` once per step of
    the busy ranks' epoch, so every rank runs the same number of steps (and collectives)."""

    def __init__(self, sampler: GlobalBatchSampler):
        self.sampler = sampler

    def __len__(self) -> int:
        return len(self.sampler)

    def __iter__(self):
        for _ in range(len(self.sampler)):
            yield None
