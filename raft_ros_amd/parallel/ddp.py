"""Multi-GPU data parallelism: one process per GPU, DDP over RCCL (xGMI).

Replaces the reference's single-process ``nn.DataParallel`` (train.py:138), which
broadcasts all 5.26 M parameters to every replica, scatters inputs and gathers
all 12 full-resolution flow predictions to GPU 0 *every step* (SURVEY.md 2.5).
Here each rank keeps its own replica; the only per-step collective is the
fp32 gradient all-reduce (~21 MB for RAFT-base): by default one packed all-reduce
after the backward (:func:`data_parallel`, parallel/grad_sync.py), or torch's
DistributedDataParallel with bucketed all-reduces (``impl="ddp"``, :func:`wrap_model`).
On ROCm the ``"nccl"`` backend is RCCL.  CPU runs (tests) use ``gloo``.

Rendezvous always uses 127.0.0.1 unless MASTER_ADDR says otherwise.
"""
from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass
from typing import Dict

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


DEFAULT_TIMEOUT_S = 600.0


def collective_timeout() -> datetime.timedelta:
    """Failure detection: a collective that does not complete within ``RAFT_DIST_TIMEOUT``
    seconds (default 600) raises on the ranks that are still alive instead of hanging the
    job forever (a dead or stuck peer; see utils/fault.py for the injection hooks)."""
    return datetime.timedelta(seconds=float(os.environ.get("RAFT_DIST_TIMEOUT", DEFAULT_TIMEOUT_S)))


def process_group_kwargs(backend: str) -> dict:
    """Options of the per-GPU process group.

    * ``timeout``: :func:`collective_timeout` (failure detection);
    * RCCL (the ``nccl`` backend on ROCm): the communicator's HIP stream is created with
      high priority, so the gradient all-reduces that DDP issues during the backward pass are
      scheduled ahead of the compute kernels queued behind them instead of waiting for a
      free slot -- over xGMI the ring all-reduce of a 10 MB bucket is short, and the step
      time is set by how early it starts.  ``RAFT_RCCL_HIGH_PRIORITY=0`` turns it off."""
    kw = {"timeout": collective_timeout()}
    if backend == "nccl" and os.environ.get("RAFT_RCCL_HIGH_PRIORITY", "1") != "0":
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        kw["pg_options"] = opts
    return kw


def init_distributed(backend: str | None = None, device_type: str | None = None) -> DistInfo:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*),
    with the collective timeout of :func:`collective_timeout`."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = (device_type or ("cuda" if torch.cuda.is_available() else "cpu")) == "cuda"
    device = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if use_cuda else "gloo")
        kw = {"device_id": device} if use_cuda else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **process_group_kwargs(backend), **kw)
    return DistInfo(rank, world, local, device)


def wrap_model(model: torch.nn.Module, info: DistInfo, bucket_cap_mb: float = 10.0, static_graph: bool = True,
               bf16_grads: bool = False):
    """DDP wrapper sized for xGMI.  RAFT-base's gradient is 21 MB fp32; the update block's
    12.5 MB are complete first (its batched weight gradients run when the last refinement
    step's backward is done, before the encoders backpropagate), so ~10 MB buckets let that
    part of the ring all-reduce run over xGMI while the encoder backward computes
    (``static_graph`` orders buckets by readiness after the first step); the encoder
    gradients follow in the last bucket.

    ``bf16_grads``: register the bf16 compression hook -- buckets are cast to bf16 for the
    ring all-reduce and back to fp32 (halves the bytes over the per-link-bound xGMI ring;
    the mean is exact up to bf16 rounding of each rank's contribution)."""
    if not info.distributed:
        return model
    kw = dict(bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True, static_graph=static_graph)
    if info.device.type == "cuda":
        kw["device_ids"] = [info.device.index]
    net = torch.nn.parallel.DistributedDataParallel(model, **kw)
    if bf16_grads:
        from torch.distributed.algorithms.ddp_comm_hooks import default_hooks

        net.register_comm_hook(None, default_hooks.bf16_compress_hook)
    return net


def data_parallel(model: torch.nn.Module, info: DistInfo, impl: str = "sync", bucket_cap_mb: float = 10.0,
                  bf16_grads: bool = False):
    """-> (module to call forward on, GradSync or None).

    ``impl="sync"`` (default): the model itself plus a :class:`~.grad_sync.GradSync` whose
    ``sync()`` the training step calls after ``backward()`` -- one packed all-reduce instead of
    DDP's per-parameter bucket copies (see parallel/grad_sync.py for why that fits RAFT).
    ``impl="ddp"``: torch's DistributedDataParallel (:func:`wrap_model`), no GradSync."""
    if not info.distributed:
        return model, None
    if impl == "ddp":
        return wrap_model(model, info, bucket_cap_mb=bucket_cap_mb, bf16_grads=bf16_grads), None
    if impl != "sync":
        raise ValueError(f"data-parallel impl {impl!r}: 'sync' or 'ddp'")
    from .grad_sync import GradSync

    return model, GradSync(model, bf16=bf16_grads)


def all_reduce_mean(values: Dict[str, float], info: DistInfo) -> Dict[str, float]:
    if not info.distributed or not values:
        return values
    keys = sorted(values)
    t = torch.tensor([float(values[k]) for k in keys], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t /= info.world_size
    return dict(zip(keys, t.tolist()))


def broadcast_buffers(model: torch.nn.Module, info: DistInfo, src: int = 0) -> None:
    """Copy every buffer (BatchNorm running statistics, ...) of ``model`` from rank ``src``.

    GradSync broadcasts parameters and buffers once, at construction; after that each rank's
    running statistics follow its own batches (and stay at their initial values on a rank
    that never had a sample).  Called before sharded validation, so every rank scores its
    share with the same statistics."""
    if not info.distributed:
        return
    with torch.no_grad():
        for b in model.buffers():
            dist.broadcast(b.data, src)


def barrier(info: DistInfo) -> None:
    if info.distributed:
        if info.device.type == "cuda":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def cleanup() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def _spawn_entry(rank, fn, nprocs, port, args):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(nprocs),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    fn(rank, *args)


def spawn(fn, nprocs: int, *args) -> None:
    """Run ``fn(rank, *args)`` in ``nprocs`` processes with torchrun-style env vars set
    (used when train.py is started without torchrun but with several --gpus).
    ``fn`` must be a module-level (picklable) function."""
    import torch.multiprocessing as mp

    mp.start_processes(_spawn_entry, args=(fn, nprocs, free_port(), args), nprocs=nprocs, start_method="spawn")
