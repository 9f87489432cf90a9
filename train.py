#!/usr/bin/env python3
"""Train RAFT -- same command line as the reference train.py (train.py:217-247).

Single GPU:        python train.py --stage chairs --gpus 0 --batch_size 8 --mixed_precision ...
Multi-GPU (DDP):   torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py --stage chairs ...
                   or  python train.py --gpus 0 1 ...   (spawns one process per listed GPU)
``--batch_size`` is the global batch, split evenly over the GPUs like the
reference's DataParallel.  Extra flags (all optional) are listed under
"MI355X options".
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--name", default="raft", help="name your experiment")
    p.add_argument("--stage", help="determines which dataset to use for training")
    p.add_argument("--restore_ckpt", help="restore checkpoint")
    p.add_argument("--small", action="store_true", help="use small model")
    p.add_argument("--validation", type=str, nargs="+")
    p.add_argument("--lr", type=float, default=0.00002)
    p.add_argument("--num_steps", type=int, default=100000)
    p.add_argument("--batch_size", type=int, default=6)
    p.add_argument("--image_size", type=int, nargs="+", default=[384, 512])
    p.add_argument("--gpus", type=int, nargs="+", default=[0, 1])
    p.add_argument("--mixed_precision", action="store_true", help="use mixed precision")
    p.add_argument("--iters", type=int, default=12)
    p.add_argument("--wdecay", type=float, default=0.00005)
    p.add_argument("--epsilon", type=float, default=1e-8)
    p.add_argument("--clip", type=float, default=1.0)
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--gamma", type=float, default=0.8, help="exponential weighting")
    p.add_argument("--add_noise", action="store_true")
    g = p.add_argument_group("MI355X options")
    g.add_argument("--amp_dtype", default="bf16", choices=["bf16", "fp16"], help="autocast dtype for --mixed_precision")
    g.add_argument("--alternate_corr", action="store_true", help="memory-efficient local correlation (trainable)")
    g.add_argument("--corr_fp32", action="store_true",
                   help="with --mixed_precision bf16: keep the correlation volume fp32-faithful (split-bf16 GEMM, "
                        "fp32 storage) like the reference (core/raft.py:102-103) instead of the bf16 volume")
    g.add_argument("--no_channels_last", dest="channels_last", action="store_false")
    g.add_argument("--no_native_encoder", dest="native_encoder", action="store_false",
                   help="encoders on PyTorch/MIOpen convs (exact fp32 training without AMP; the native fp32 "
                        "encoder runs split-bf16 GEMMs)")
    g.add_argument("--batch_split", default="balanced", choices=["balanced", "chunk"],
                   help="how the global --batch_size splits over the ranks: balanced (10 over 8 = 2,2,1,1,1,1,1,1) "
                        "or chunk (DataParallel's torch.chunk grouping: 2,2,2,2,2,0,0,0)")
    g.add_argument("--no_fused_update", dest="fused_update", action="store_false",
                   help="run the update block on PyTorch convs instead of the fused HIP kernels")
    g.add_argument("--resume", action="store_true", help="also restore optimizer/scheduler/step from <ckpt>.state.pt")
    g.add_argument("--num_workers", type=int, default=4)
    g.add_argument("--ckpt_dir", default="checkpoints")
    g.add_argument("--log_dir", default="runs")
    g.add_argument("--dataset_root", default=None, help="directory holding Sintel/, KITTI/, ... (default ./datasets)")
    g.add_argument("--dp_impl", choices=["sync", "ddp"], default="sync",
                   help="data-parallel gradient averaging: one packed all-reduce after the backward (sync, "
                        "parallel/grad_sync.py) or torch DistributedDataParallel (ddp)")
    g.add_argument("--bucket_mb", type=float, default=10.0,
                   help="DDP gradient bucket size (--dp_impl ddp)")
    g.add_argument("--seed", type=int, default=1234)
    g.add_argument("--deterministic", action="store_true",
                   help="bitwise-reproducible steps: torch.use_deterministic_algorithms + the native kernels' "
                        "atomic-free / fixed-point-atomic backward paths")
    g.add_argument("--sync_bn", action="store_true",
                   help="synchronize the context encoder's BatchNorm statistics over the DDP ranks (default: "
                        "per-rank statistics, like the reference's DataParallel replicas)")
    g.add_argument("--ddp_bf16_grads", action="store_true",
                   help="all-reduce gradients in bf16 (halves xGMI traffic)")
    g.add_argument("--graph", action="store_true",
                   help="replay each training step as captured HIP graph(s) (static crops; the gradient "
                        "all-reduce runs between two graphs; no host issue per step).  Off by default: since "
                        "the native clip + AdamW op the eager step is GPU-bound down to batch 1 and keeps its "
                        "stream priorities (368x768 batch 1: eager 134.0 vs graph 124.2 pairs/s, batch 8 at "
                        "368x496: 471 vs 436; profiles/r6s_*, r6c_*)")
    g.add_argument("--synthetic_pool", type=int, default=8,
                   help="--stage synthetic: batches per rank in the device-resident pool that is replayed "
                        "(a throughput check: only pool x batch distinct pairs); 0 = 100000 distinct pairs "
                        "generated by CPU DataLoader workers (~200 pairs/s on one MI355X), globally aligned")
    g.add_argument("--profile_dir", default=None, help="capture a torch.profiler trace of steps 5-7 here")
    return p


def _main(args) -> str:
    from raft_ros_amd.train.trainer import train

    rank = int(os.environ.get("RANK", "0"))
    torch.manual_seed(args.seed + rank)
    # the same numpy stream on every rank: --add_noise draws ONE sigma per global batch, as the
    # reference does (train.py:167-170); per-rank augmentation has its own generators
    np.random.seed(args.seed)
    if getattr(args, "deterministic", False):
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.backends.cudnn.benchmark = False
    os.makedirs(args.ckpt_dir, exist_ok=True)
    return train(args)


def _spawned(rank: int, args) -> None:
    os.environ["LOCAL_RANK"] = str(args.gpus[rank])
    _main(args)


def check_gpus(gpus, ndev=None) -> None:
    """Refuse ``--gpus`` ids the node does not have (the reference default ``--gpus 0 1``,
    train.py:229, would otherwise start a rank that dies on ``cuda:1`` of a 1-GPU box).
    ``torch.cuda.device_count()`` does not initialise HIP, so this is safe before spawning.
    Without a GPU (CPU runs, tests) the ids are not checked.  Under torchrun the world size,
    not ``--gpus``, decides the ranks."""
    if "WORLD_SIZE" in os.environ:
        return
    ndev = torch.cuda.device_count() if ndev is None else ndev
    if ndev == 0:
        return
    bad = [g for g in gpus if not 0 <= g < ndev]
    if bad or len(set(gpus)) != len(gpus):
        raise SystemExit(f"train.py: --gpus {' '.join(map(str, gpus))} but this node has {ndev} visible GPU(s) "
                         f"(ids 0..{ndev - 1}); pass e.g. --gpus {' '.join(map(str, range(min(len(gpus), ndev))))}")


def main(argv=None):
    args = build_parser().parse_args(argv)
    if args.dataset_root:
        os.environ["RAFT_DATASET_ROOT"] = args.dataset_root
    check_gpus(args.gpus)
    if "WORLD_SIZE" not in os.environ and len(args.gpus) > 1 and torch.cuda.is_available():
        from raft_ros_amd.parallel.ddp import spawn

        spawn(_spawned, len(args.gpus), args)
        return None
    if "LOCAL_RANK" not in os.environ and torch.cuda.is_available():
        os.environ["LOCAL_RANK"] = str(args.gpus[0])
    return _main(args)


if __name__ == "__main__":
    main()
