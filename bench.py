#!/usr/bin/env python3
"""Training-throughput benchmark: RAFT-base, FlyingChairs-shaped synthetic pairs.

Config (BASELINE.json config #2/#3): RAFT base, 368x496 crops, 12 GRU
iterations, bf16 autocast, full training step = forward + sequence loss +
backward + grad-clip + fused AdamW + OneCycle step.  Weak scaling: the
per-GPU batch (``--batch``, default 8 = train_mixed.sh's chairs batch) is fixed
and the global batch is ``batch * N``.  Multi-GPU runs are one process per GPU
(torchrun) with DistributedDataParallel over RCCL.

Prints ONE JSON line on rank 0 (see README "bench contract").  ``value`` is
whole-job image pairs per second.  ``vs_baseline`` divides by the eager
PyTorch baseline of the reference algorithm measured on the same MI355X
("measured" row), when present.

    python bench.py                      # 1 GPU, defaults
    python bench.py --impl reference     # the reference's eager op sequence (baseline)
    python bench.py --gpus 8             # spawns 8 rank processes itself (no torchrun needed)
    torchrun --nproc-per-node 8 bench.py --gpus 8

Launch contract: under torchrun (WORLD_SIZE set) every process is one rank and
``--gpus`` must equal WORLD_SIZE.  Without WORLD_SIZE and ``--gpus N > 1`` the
parent process starts N rank processes with ``torch.multiprocessing`` (spawn)
BEFORE touching the GPU, and exits with the first non-zero rank exit code.
``n_gpus`` in the JSON is always the real world size.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from argparse import Namespace

import torch
import torch.distributed as dist

METRIC = "image-pairs/sec training + Sintel-clean EPE, RAFT base at 1/2/4/8 MI355X"
# Eager PyTorch baseline of the reference algorithm on 1x MI355X (pairs/s), see BASELINE.md
BASELINE_PAIRS_PER_SEC = 96.593  # measured r2 (profiles/r2_bench_ref_bench_v3.json): bench.py --impl reference, bf16, batch 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="per-GPU batch (weak scaling)")
    ap.add_argument("--global_batch", type=int, default=0,
                    help="> 0: strong scaling at this GLOBAL batch, split over the ranks as the trainer does "
                         "(parallel/batching.py: the reference's DataParallel semantics; train_standard.sh on 8 "
                         "GPUs = --global_batch 6 -> 1,1,1,1,1,1,0,0 with loss weights, idle ranks still in the "
                         "all-reduce and the optimizer step); --batch is then ignored")
    ap.add_argument("--image_size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--impl", choices=["native", "reference"], default="native")
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--amp_dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--fp32", action="store_true",
                    help="no autocast (mixed_precision=False): the reference's default for demo.py / evaluate.py / "
                         "the ROS node and train_standard.sh")
    ap.add_argument("--corr_fp32", action="store_true",
                    help="bf16 AMP with the reference's fp32-faithful correlation volume (core/raft.py:102-103)")
    ap.add_argument("--lr", type=float, default=4e-4)
    # ~10 MB buckets: the update-block gradients (12.5 MB, ready first -- batched wgrads run
    # before the encoders' backward) all-reduce over xGMI while the encoders backpropagate
    ap.add_argument("--bucket_mb", type=float, default=10.0, help="DDP bucket size (--dp_impl ddp)")
    ap.add_argument("--dp_impl", choices=["sync", "ddp"], default="sync",
                    help="N>1 gradient averaging: one packed all-reduce after the backward "
                         "(parallel/grad_sync.py) or torch DistributedDataParallel")
    ap.add_argument("--no_fused", action="store_true", help="update block on PyTorch/MIOpen convs")
    ap.add_argument("--mode", choices=["train", "infer"], default="train",
                    help="infer: forward-only test_mode passes (BASELINE config #5: --image_size 1080 1920 --iters 32)")
    ap.add_argument("--alternate_corr", action="store_true", help="memory-efficient local correlation (config #4)")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=None,
                    help="replay the step as captured HIP graph(s) (train: fwd+loss+bwd+clip+AdamW, grads "
                         "all-reduced between two graphs when N>1; infer: the forward). Default: on for infer; "
                         "off for train, where the step is GPU-bound and eager keeps more of the multi-stream overlap "
                         "(graph 394.6 vs eager 402.0 pairs/s on MI355X; 1080p inference 60.9 graph vs 60.7 eager, profiles/r3_graph_vs_eager.log)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: gloo-backend plumbing check of the launch path only (tests), never a measurement")
    return ap.parse_args()


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _rank_entry(rank, nprocs, port, argv):
    """Child process of ``python bench.py --gpus N`` (no torchrun): one rank per GPU."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(nprocs),
                      LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = [sys.argv[0]] + list(argv)
    run(parse())


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # spawn the ranks before anything initialises HIP in this process
        # (torch.cuda.device_count() does not initialise the runtime)
        ndev = torch.cuda.device_count() if args.device == "cuda" else args.gpus
        if ndev < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but only {ndev} GPU(s) visible")
        import torch.multiprocessing as mp

        from raft_ros_amd.parallel.ddp import free_port

        mp.start_processes(_rank_entry, args=(args.gpus, free_port(), sys.argv[1:]), nprocs=args.gpus,
                           start_method="spawn")
        return 0
    return run(args)


def _allreduce_ms(model, device, world, reps: int = 10) -> float:
    """Time of one all-reduce of a gradient-sized fp32 buffer (what DDP moves per step)."""
    if world <= 1:
        return 0.0
    n = sum(p.numel() for p in model.parameters() if p.requires_grad)
    buf = torch.ones(n, device=device, dtype=torch.float32)
    for _ in range(3):
        dist.all_reduce(buf)
    _sync(device)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(buf)
    _sync(device)
    t = torch.tensor([(time.perf_counter() - t0) / reps], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return 1000.0 * float(t.item())


def _paths(model, image, args):
    """(encoder path, update-block path) the model's dispatch takes for this run's mode."""
    if args.impl == "reference":
        return "reference", "reference"
    amp = not args.fp32
    grad = args.mode == "train"
    with torch.set_grad_enabled(grad):
        enc = "native-hip" if model._use_native_encoders(image, amp) else "module"
        if amp:
            upd = ("fused-hip-" + args.amp_dtype) if model._use_fused(image, amp) else "module"
        elif grad:
            upd = "split-fp32-hip" if model._use_split_train(image, amp) else "module"
        else:
            upd = "split-fp32-hip" if model._use_split(image, amp) else "module"
    if enc == "native-hip" and not amp:
        enc = "native-hip-split-fp32"
    return enc, upd


def _corr_volume(model, args, device):
    """Storage precision of the dense correlation volume the model builds (its own rule in
    RAFT.forward), or None when no native dense volume is built (the reference implementation,
    --alternate_corr)."""
    if args.impl == "reference" or args.alternate_corr:
        return None
    amp = not args.fp32
    bf16_amp = amp and device.type == "cuda" and model.amp_dtype == torch.bfloat16
    return "fp32" if (not bf16_amp or bool(getattr(model.args, "corr_fp32", False))) else "bf16"


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if "WORLD_SIZE" in os.environ and args.gpus != world and rank == 0:
        print(f"bench.py: warning: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the real world size",
              file=sys.stderr, flush=True)
    if args.device == "cuda":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        if distributed:
            from raft_ros_amd.parallel.ddp import process_group_kwargs

            # high-priority RCCL stream: DDP's bucket all-reduces overtake queued backward kernels
            dist.init_process_group("nccl", device_id=device, **process_group_kwargs("nccl"))
    else:
        device = torch.device("cpu")
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(world, 1)))
        if distributed:
            dist.init_process_group("gloo")

    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.ops import _ext
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.optim import fetch_optimizer
    from raft_ros_amd.train.trainer import init_idle_scaler

    _ext.set_backend(args.impl)
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(1234 + rank)
    margs = Namespace(small=args.small, mixed_precision=not args.fp32, amp_dtype=args.amp_dtype,
                      alternate_corr=args.alternate_corr,
                      dropout=0.0, channels_last=args.impl == "native",
                      fused_update=not args.no_fused, corr_fp32=args.corr_fp32)
    model = RAFT(margs).to(device)
    if args.impl == "native":
        model = model.to(memory_format=torch.channels_last)
    model.train()
    oargs = Namespace(lr=args.lr, wdecay=1e-4, epsilon=1e-8, num_steps=100000)
    train_graph = (bool(args.graph) and args.mode == "train" and args.impl == "native" and args.amp_dtype == "bf16"
                   and not args.fp32)
    gsync = None
    if distributed and not train_graph and args.dp_impl == "ddp":
        ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local] if device.type == "cuda" else None,
                                                        bucket_cap_mb=args.bucket_mb,
                                                        gradient_as_bucket_view=True, static_graph=True)
    else:
        ddp = model
        if distributed and not train_graph:
            from raft_ros_amd.parallel.grad_sync import GradSync

            gsync = GradSync(model)
    # eager bf16 / fp32 steps: clip + AdamW as one native op (ops/optim.py), as the trainer runs it
    native_opt = args.impl == "native" and not train_graph and args.mode == "train" and (
        args.fp32 or args.amp_dtype == "bf16") and device.type == "cuda"
    optimizer, scheduler = fetch_optimizer(oargs, model, capturable=train_graph, clip=1.0 if native_opt else None)
    native_opt = not isinstance(optimizer, torch.optim.AdamW)
    scaler = torch.amp.GradScaler("cuda", enabled=args.amp_dtype == "fp16" and not args.fp32 and device.type == "cuda")

    H, W = args.image_size
    # strong scaling (--global_batch): this rank's share of the global batch and its loss weight
    sizes = None
    if args.global_batch > 0:
        from raft_ros_amd.parallel.batching import loss_weight, rank_batch_sizes

        if args.mode != "train" or train_graph or (distributed and args.dp_impl == "ddp"):
            raise SystemExit("bench.py: --global_batch measures eager training with --dp_impl sync")
        sizes = rank_batch_sizes(args.global_batch, world)
        args.batch = sizes[rank]
    weight = loss_weight(sizes, rank) if sizes is not None else 1.0
    idle = args.batch == 0
    pool = [synthetic_batch(max(args.batch, 1), H, W, seed=rank * 97 + i, device=device)
            for i in range(2 if H * W > 1e6 else 4)]

    if args.mode == "infer":
        from raft_ros_amd.runtime import GraphedRAFT

        model.eval()
        runner = GraphedRAFT(model, iters=args.iters, enabled=args.graph is not False)

        @torch.inference_mode()
        def step(i):
            i1, i2, flow, valid = pool[i % len(pool)]
            _, flow_up = runner(i1, i2)
            return flow_up.new_zeros(()), {"epe": (flow_up - flow).norm(dim=1).mean()}
    else:
        step = None

    params = [p for p in model.parameters() if p.requires_grad]  # not re-walked per step (host time)

    def train_step(i):
        i1, i2, flow, valid = pool[i % len(pool)]
        optimizer.zero_grad(set_to_none=True)
        if idle:  # no sample of the global batch here: zero gradients into the all-reduce
            loss = torch.zeros((), device=device)
            metrics = {"epe": torch.zeros((), device=device)}
            init_idle_scaler(scaler, device)
        else:
            preds = ddp(i1, i2, iters=args.iters)
            loss, metrics = sequence_loss(preds, flow, valid, gamma=0.8)
            if weight != 1.0:
                loss = loss * weight
            scaler.scale(loss).backward()
        if gsync is not None:
            gsync.sync()
        if native_opt:
            optimizer.step()  # clip (1.0) + AdamW
        else:
            scaler.unscale_(optimizer)
            torch.nn.utils.clip_grad_norm_(params, 1.0)
            scaler.step(optimizer)
            scaler.update()
        scheduler.step()
        return loss, metrics

    if train_graph:
        from raft_ros_amd.runtime import GraphedTrainStep

        runner = GraphedTrainStep(model, optimizer, sequence_loss, iters=args.iters, clip=1.0, gamma=0.8)

        def graph_step(i):
            i1, i2, flow, valid = pool[i % len(pool)]
            loss, metrics, _ = runner(i1, i2, flow, valid)
            scheduler.step()
            return loss, metrics

        step = graph_step
    step = step or train_step
    # the step on a high-priority stream (ops/streams.py step_stream; RAFT_HP_MAIN=0 disables):
    # the refinement loop's critical path is dispatched ahead of the side / tail streams' kernels
    if args.mode == "train" and not train_graph:
        from raft_ros_amd.ops.streams import step_context

        plain_step = step

        def step(i):  # noqa: F811
            with step_context(device):
                return plain_step(i)
    from raft_ros_amd.ops.streams import LeadLimiter

    # the trainer's bound on how far the host runs ahead (RAFT_MAX_LEAD=0: unbounded)
    lead = LeadLimiter(max_lead=int(os.environ.get("RAFT_MAX_LEAD", "2")))
    for i in range(args.warmup):
        loss, metrics = step(i)
        lead.step_done(device)
    _sync(device)
    if distributed:
        dist.barrier()
    _sync(device)
    # RAFT_BENCH_STEP_TIMES=1: per-step GPU time (events on the current stream) to stderr
    step_ev = [] if (os.environ.get("RAFT_BENCH_STEP_TIMES") == "1" and device.type == "cuda") else None
    t0 = time.perf_counter()
    for i in range(args.steps):
        if step_ev is not None:
            step_ev.append(torch.cuda.Event(enable_timing=True))
            step_ev[-1].record()
        loss, metrics = step(args.warmup + i)
        lead.step_done(device)
    if step_ev is not None:
        step_ev.append(torch.cuda.Event(enable_timing=True))
        step_ev[-1].record()
    _sync(device)
    if step_ev is not None:
        ms = [a.elapsed_time(b) for a, b in zip(step_ev, step_ev[1:])]
        print("step ms: " + " ".join(f"{v:.2f}" for v in ms), file=sys.stderr, flush=True)
    if distributed:
        dist.barrier()
    _sync(device)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ar_ms = _allreduce_ms(model, device, world)
    enc_path, upd_path = _paths(model, pool[0][0], args)
    pairs = (args.global_batch if sizes is not None else args.batch * world) * args.steps
    value = pairs / elapsed
    if rank == 0:
        out = {
            "metric": METRIC if args.mode == "train" else "image-pairs/sec inference (test_mode), RAFT",
            "value": round(value, 3),
            "unit": "image-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if sizes is not None else "weak",
            "vs_baseline": (round(value / (BASELINE_PAIRS_PER_SEC * world), 3)
                            if BASELINE_PAIRS_PER_SEC and args.impl == "native" and args.mode == "train" and not args.fp32
                            and not args.small and not args.alternate_corr and (H, W) == (368, 496)
                            and args.iters == 12 and args.batch == 8 and sizes is None else None),
            "dtype": args.amp_dtype if device.type == "cuda" and not args.fp32 else "fp32",
            "data": "synthetic (textured pairs warped by known smooth flow; random-init weights)",
            "config": {
                "model": "RAFT-small" if args.small else "RAFT-base",
                "global_batch": args.global_batch if sizes is not None else args.batch * world,
                "rank_batches": sizes,
                "seq_len": args.iters,
                "image_size": [H, W],
                "iters": args.iters,
                "parallelism": f"dp{world}",
                "dp_impl": (args.dp_impl if world > 1 else None),
                "impl": args.impl,
                # the code paths that actually ran (decided by the model's own dispatch rules)
                "fused_update": upd_path not in ("module", "reference"),
                "update_path": upd_path,
                "encoder_path": enc_path,
                "corr_volume": _corr_volume(model, args, device),
                "mode": args.mode,
                "alternate_corr": args.alternate_corr,
                "hip_graph": bool(train_graph or (args.graph is not False and args.mode == "infer")),
                "optimizer": "native clip+AdamW (2 launches)" if native_opt else "torch clip_grad_norm_ + AdamW",
            },
            "final_loss": round(float(loss.item()), 4),
            "epe_synthetic": round(float(metrics["epe"].item()), 4),
            "peak_mem_gb": (round(torch.cuda.max_memory_allocated(device) / 2**30, 2)
                            if device.type == "cuda" else None),
            "allreduce_ms": round(ar_ms, 3),
        }
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
