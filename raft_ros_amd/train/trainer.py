"""RAFT training loop (reference train.py:136-214), MI355X / multi-GPU edition.

Same schedule semantics as the reference: AdamW + OneCycle (``fetch_optimizer``),
sequence loss with ``args.gamma``, optional Gaussian input noise
(``--add_noise``, sigma ~ U(0, 5)), gradient clipping to ``args.clip``, BatchNorm
frozen for every stage except chairs (re-applied after validation), a weights
checkpoint every ``VAL_FREQ`` steps followed by validation, and a final
``checkpoints/<name>.pth`` -- in the reference's ``module.``-prefixed format.

MI355X-specific:

* one process per GPU with DDP over RCCL (torchrun, or ``--gpus 0 1 ...``
  which spawns the ranks itself); ``--batch_size`` stays the GLOBAL batch, split
  exactly over the ranks (``parallel/batching.py``: 10 over 8 ranks trains 10
  samples per step, each rank's loss weighted by its share; idle ranks of a
  batch smaller than the world contribute zero gradients);
* bf16 autocast by default for ``--mixed_precision`` (``--amp_dtype fp16``
  restores the reference's fp16 + GradScaler);
* channels-last model, fused AdamW, loss metrics kept on the device;
* non-finite-loss guard (the step is skipped and counted) and an exact-resume
  sidecar ``<name>.state.pt`` next to every checkpoint.
"""
from __future__ import annotations

import os
import time
from argparse import Namespace

import numpy as np
import torch

from ..data.datasets import fetch_dataloader
from ..eval.validate import run_validation
from ..models import RAFT
from ..ops.streams import LeadLimiter, step_context
from ..parallel import ddp
from ..parallel.batching import check_sync_bn, loss_weight, rank_batch_sizes
from ..utils import checkpoint, fault
from ..utils.profiling import maybe_profiler, trace_range
from .logger import Logger
from .loss import METRIC_KEYS, sequence_loss
from .optim import count_parameters, fetch_optimizer

VAL_FREQ = 5000


def _infinite(loader, sampler_epoch=None):
    epoch = 0
    while True:
        if sampler_epoch is not None:
            sampler_epoch(epoch)
        for batch in loader:
            yield batch
        epoch += 1


def _dummy_batch(image_size):
    """One all-zero sample (weight 0): an idle rank's forward under torch DDP."""
    h, w = int(image_size[0]), int(image_size[1])
    return (torch.zeros(1, 3, h, w), torch.zeros(1, 3, h, w), torch.zeros(1, 2, h, w), torch.zeros(1, h, w))


def init_idle_scaler(scaler, device) -> None:
    """Initialise an enabled GradScaler's scale on a rank that has no sample this step.

    ``GradScaler.scale()`` creates the scale tensor lazily; a GradSync rank without a sample
    never calls it, and ``unscale_`` would then fail ('_scale is None') while the other ranks
    wait in the next all-reduce.  Scaling a zero keeps the scale at its current value on every
    rank (the update after ``step`` sees the same all-reduced gradients everywhere)."""
    if scaler.is_enabled():
        scaler.scale(torch.zeros((), device=device))


def train(args: Namespace, on_finish=None) -> str:
    info = ddp.init_distributed()
    args.rank, args.world_size = info.rank, info.world_size
    dev = info.device
    # the global batch split over the ranks, and this rank's loss weight (b_r * W / B: the
    # AVG all-reduce of the weighted gradients is the full-batch gradient)
    sizes = rank_batch_sizes(args.batch_size, info.world_size, getattr(args, "batch_split", "balanced"))
    weight = loss_weight(sizes, info.rank)
    if info.distributed and info.is_main:
        print(f"global batch {args.batch_size} over {info.world_size} ranks: {sizes}")
    if getattr(args, "sync_bn", False) and info.distributed:
        check_sync_bn(sizes)

    model = RAFT(args)
    if info.is_main:
        print("Parameter Count: %d" % count_parameters(model))
    if args.restore_ckpt is not None:
        checkpoint.load_weights(model, args.restore_ckpt, strict=False)
    model = model.to(dev)
    if dev.type == "cuda" and getattr(args, "channels_last", True):
        model = model.to(memory_format=torch.channels_last)
    model.train()
    if getattr(args, "sync_bn", False) and info.distributed:
        # global-batch BatchNorm statistics for the context encoder (parallel/sync_bn.py); the
        # default keeps the reference's per-replica statistics (DataParallel, train.py:138)
        from ..parallel.sync_bn import convert_sync_bn

        convert_sync_bn(model.cnet)
    if args.stage != "chairs":
        model.freeze_bn()
    use_scaler = bool(args.mixed_precision) and getattr(args, "amp_dtype", "bf16") == "fp16" and dev.type == "cuda"
    # --graph: the whole step replayed as HIP graph(s) (runtime/train_graph.py), which does its own
    # flat-buffer gradient all-reduce between two graphs -- no GradSync / DDP wrapper
    use_graph = bool(getattr(args, "graph", False)) and dev.type == "cuda" and not use_scaler
    if use_graph:
        net, gsync = model, None
    else:
        net, gsync = ddp.data_parallel(model, info, impl=getattr(args, "dp_impl", "sync"),
                                       bucket_cap_mb=getattr(args, "bucket_mb", 10.0),
                                       bf16_grads=getattr(args, "ddp_bf16_grads", False))

    args.device = str(dev)  # batched augmentation runs on the rank's device
    train_loader = fetch_dataloader(args)
    # without a GradScaler the eager clip + AdamW step is one native op (ops/optim.py ClipAdamW);
    # the graphed step captures torch's capturable fused AdamW (device lr and step count)
    optimizer, scheduler = fetch_optimizer(args, model, capturable=use_graph,
                                           clip=None if (use_scaler or use_graph) else args.clip)
    native_opt = not isinstance(optimizer, torch.optim.AdamW)
    runner = None
    if use_graph:
        from ..runtime import GraphedTrainStep

        w = 0.0 if sizes[info.rank] == 0 else weight  # an idle rank replays a zero-weight dummy sample

        def weighted_loss(preds, flow, valid, gamma):
            loss, m = sequence_loss(preds, flow, valid, gamma)
            if w != 1.0:
                loss = loss * w
                m = {k: v * w for k, v in m.items()}
            return loss, m

        runner = GraphedTrainStep(model, optimizer, weighted_loss, iters=args.iters, clip=args.clip, gamma=args.gamma)
    scaler = torch.amp.GradScaler("cuda", enabled=use_scaler)
    logger = Logger(model, scheduler, log_dir=os.path.join(args.log_dir, args.name), enabled=info.is_main,
                    pairs_per_step=args.batch_size,
                    reduce_fn=(lambda m: ddp.all_reduce_mean(m, info)) if info.distributed else None)

    total_steps = 0
    if getattr(args, "resume", False) and args.restore_ckpt is not None:
        st = checkpoint.load_state(checkpoint.state_path(args.restore_ckpt), optimizer, scheduler, scaler)
        if st is not None:
            total_steps = st
            logger.total_steps = st
            if info.is_main:
                print(f"resumed at step {st}")

    set_epoch = None
    for smp in (train_loader, getattr(train_loader, "batch_sampler", None), getattr(train_loader, "sampler", None)):
        if hasattr(smp, "set_epoch"):
            set_epoch = smp.set_epoch
            break
    skipped = torch.zeros((), device=dev)
    fused_opt = bool(optimizer.defaults.get("fused"))
    injector = fault.Injector.from_env(info.rank)  # RAFT_FAULT_INJECT (tests only)
    t0 = time.perf_counter()
    lead = LeadLimiter(max_lead=2)  # host at most 2 steps ahead of the GPU (ops/streams.py)
    prof = maybe_profiler(getattr(args, "profile_dir", None))
    profiler = prof.__enter__()
    clip_params = [p for p in model.parameters() if p.requires_grad]  # walked once, not per step

    def _after_step(step: int) -> int:
        """Checkpoint + validation every VAL_FREQ steps (reference train.py:186-199); -> step + 1."""
        total_steps = step
        if total_steps % VAL_FREQ == VAL_FREQ - 1:
            path = os.path.join(args.ckpt_dir, "%d_%s.pth" % (total_steps + 1, args.name))
            if info.is_main:
                checkpoint.save_weights(model, path)
                checkpoint.save_state(checkpoint.state_path(path), optimizer, scheduler, scaler, total_steps + 1)
            # validation is sharded over the ranks and each rank scores its share with its own
            # BatchNorm running statistics: take rank 0's (the reference's replica-0 statistics,
            # train.py:138), which also covers ranks that sat idle and never updated theirs
            ddp.broadcast_buffers(model, info)
            results = run_validation(model, args.validation, rank=info.rank, world=info.world_size)
            logger.write_dict(results)
            model.train()
            if args.stage != "chairs":
                model.freeze_bn()
            ddp.barrier(info)
        return total_steps + 1

    for data_blob in _infinite(train_loader, set_epoch):
        injector.before_step(total_steps)
        if runner is not None:
            # --graph: the step is one graph replay (two around the gradient all-reduce); an idle
            # rank replays its zero-weight dummy sample to stay in the collective
            if data_blob is None:
                data_blob = _dummy_batch(args.image_size)
            image1, image2, flow, valid = [x.to(dev, non_blocking=True) for x in data_blob]
            if args.add_noise:
                stdv = np.random.uniform(0.0, 5.0)  # drawn on every rank: same RNG stream
                image1 = (image1 + stdv * torch.randn_like(image1)).clamp(0.0, 255.0)
                image2 = (image2 + stdv * torch.randn_like(image2)).clamp(0.0, 255.0)
            _, metrics, _ = runner(image1, image2, flow, valid)
            scheduler.step()  # writes the captured optimizer's device lr
            logger.push(metrics)
            if profiler is not None:
                profiler.step()
            lead.step_done(dev)
            total_steps = _after_step(total_steps)
            if total_steps > args.num_steps:
                break
            continue
        # the step on the high-priority step stream (ops/streams.py; RAFT_HP_MAIN=0 disables)
        with step_context(dev):
            optimizer.zero_grad(set_to_none=True)
            idle = data_blob is None  # no sample of the global batch on this rank
            if idle and gsync is None:
                # torch DDP needs every rank in the backward: a zero-weight dummy sample
                data_blob = _dummy_batch(args.image_size)
            if args.add_noise:
                stdv = np.random.uniform(0.0, 5.0)  # drawn on every rank: same RNG stream
            if idle and gsync is not None:
                metrics = {k: torch.zeros((), device=dev) for k in METRIC_KEYS}
                # no loss to scale here, but GradScaler.unscale_ below needs its scale tensor:
                # the idle rank must run the same unscale / step / update as the busy ones
                init_idle_scaler(scaler, dev)
            else:
                image1, image2, flow, valid = [x.to(dev, non_blocking=True) for x in data_blob]
                if args.add_noise:
                    image1 = (image1 + stdv * torch.randn_like(image1)).clamp(0.0, 255.0)
                    image2 = (image2 + stdv * torch.randn_like(image2)).clamp(0.0, 255.0)

                with trace_range("forward"):
                    flow_predictions = net(image1, image2, iters=args.iters)
                    loss, metrics = sequence_loss(flow_predictions, flow, valid, args.gamma)
                    loss = injector.on_loss(total_steps, loss)
                    if weight != 1.0 or idle:
                        loss = loss * (0.0 if idle else weight)
                        metrics = {k: v * (0.0 if idle else weight) for k, v in metrics.items()}
                with trace_range("backward"):
                    scaler.scale(loss).backward()
            if gsync is not None:
                with trace_range("grad_sync"):
                    gsync.sync()
            scaler.unscale_(optimizer)
            if native_opt:
                # clip + AdamW in two launches; a non-finite norm skips the update on device and
                # counts in `skipped` (no host sync)
                optimizer.step(skipped=skipped)
            elif use_scaler:
                torch.nn.utils.clip_grad_norm_(clip_params, args.clip)
                scaler.step(optimizer)  # GradScaler already skips non-finite steps
                scaler.update()
            else:
                gnorm = torch.nn.utils.clip_grad_norm_(clip_params, args.clip)
                # failure guard without a host sync: a non-finite gradient norm (identical on all
                # ranks after the all-reduce) turns the fused AdamW update into a no-op on device
                bad = (~torch.isfinite(gnorm)).float()
                skipped += bad
                if fused_opt:
                    optimizer.found_inf = bad
                    optimizer.step()
                    optimizer.found_inf = None
                elif not bool(bad):
                    optimizer.step()
            scheduler.step()
            logger.push(metrics)
            if profiler is not None:
                profiler.step()
        lead.step_done(dev)
        total_steps = _after_step(total_steps)
        if total_steps > args.num_steps:
            break

    prof.__exit__(None, None, None)
    nskip = runner.skipped if runner is not None and runner.skipped is not None else skipped
    if info.is_main:
        dt = time.perf_counter() - t0
        print(f"trained {total_steps} steps in {dt:.1f}s ({args.batch_size * total_steps / dt:.2f} "
              f"pairs/s, {int(nskip.item())} non-finite steps skipped)")
    logger.close()
    path = os.path.join(args.ckpt_dir, "%s.pth" % args.name)
    if info.is_main:
        checkpoint.save_weights(model, path)
        checkpoint.save_state(checkpoint.state_path(path), optimizer, scheduler, scaler, total_steps)
    if on_finish is not None:  # test hook: inspect every rank's final model
        on_finish(model, info)
    ddp.barrier(info)
    ddp.cleanup()
    return path
