"""Exact global-batch semantics under one process per rank (parallel/batching.py).

The reference's ``--batch_size`` is the global batch that nn.DataParallel splits over its
replicas (train.py:138, train_standard.sh: batch 10 and 6 on 2 GPUs).  Here the batch is split
over gloo ranks -- unevenly when it does not divide the world size, with idle ranks when it is
smaller -- and each rank's loss is weighted by its share, so the averaged gradient is the
gradient of the full batch.  The last test runs the real trainer (train.py's parser +
trainer.train) on 2 ranks and checks replica sync and rank-0-only checkpoint writes."""
import os
import tempfile
from argparse import Namespace

import pytest
import torch
import torch.multiprocessing as mp

from raft_ros_amd.parallel import ddp
from raft_ros_amd.parallel.batching import GlobalBatchSampler, loss_weight, rank_batch_sizes


def test_rank_batch_sizes():
    assert rank_batch_sizes(10, 8) == [2, 2, 1, 1, 1, 1, 1, 1]
    assert rank_batch_sizes(6, 8) == [1, 1, 1, 1, 1, 1, 0, 0]
    assert rank_batch_sizes(6, 4) == [2, 2, 1, 1]
    assert rank_batch_sizes(10, 2) == [5, 5]
    # DataParallel's scatter (torch.chunk)
    assert rank_batch_sizes(10, 8, "chunk") == [2, 2, 2, 2, 2, 0, 0, 0]
    assert rank_batch_sizes(6, 4, "chunk") == [2, 2, 2, 0]
    assert rank_batch_sizes(6, 8, "chunk") == [1, 1, 1, 1, 1, 1, 0, 0]
    assert [len(c) for c in torch.arange(10).chunk(8)] == [s for s in rank_batch_sizes(10, 8, "chunk") if s]
    for B in range(1, 13):
        for W in (1, 2, 3, 4, 8):
            for pol in ("balanced", "chunk"):
                s = rank_batch_sizes(B, W, pol)
                assert len(s) == W and sum(s) == B and min(s) >= 0
                assert abs(sum(b / B * 1.0 for b in s) - 1.0) < 1e-12
                assert abs(sum(loss_weight(s, r) for r in range(W)) / W - 1.0) < 1e-12


def test_global_batch_sampler_disjoint_and_aligned():
    sizes = rank_batch_sizes(10, 8)
    samplers = [GlobalBatchSampler(95, sizes, r, seed=3) for r in range(8)]
    assert all(len(s) == 9 for s in samplers)  # 95 // 10 steps on every rank (drop_last)
    for epoch in (0, 1):
        for s in samplers:
            s.set_epoch(epoch)
        its = [list(s) for s in samplers]
        for step in range(9):
            parts = [its[r][step] for r in range(8)]
            assert [len(p) for p in parts] == sizes
            flat = sum(parts, [])
            assert len(set(flat)) == 10  # the ranks' slices are disjoint
        if epoch == 0:
            first = its[0][0]
    samplers[0].set_epoch(0)
    assert list(samplers[0])[0] == first  # the order is a function of (seed, epoch) only
    samplers[0].set_epoch(1)
    assert list(samplers[0])[0] != first


def _batch(B):
    from raft_ros_amd.data.synthetic import synthetic_batch

    return synthetic_batch(B, 128, 128, max_disp=4, seed=11)


def _worker(rank, world, port, tmpdir, B, impl):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.trainer import _dummy_batch

    info = ddp.init_distributed(device_type="cpu")
    torch.manual_seed(0)
    model = RAFT(Namespace(small=True, mixed_precision=False))
    net, gsync = ddp.data_parallel(model, info, impl=impl)
    sizes = rank_batch_sizes(B, world)
    lo = sum(sizes[:rank])
    i1, i2, flow, valid = _batch(B)
    if sizes[rank] > 0:
        sl = slice(lo, lo + sizes[rank])
        loss, _ = sequence_loss(net(i1[sl], i2[sl], iters=2), flow[sl], valid[sl])
        (loss * loss_weight(sizes, rank)).backward()
    elif gsync is None:  # torch DDP: the trainer's zero-weight dummy sample
        d = _dummy_batch((128, 128))
        loss, _ = sequence_loss(net(d[0], d[1], iters=2), d[2], d[3])
        (loss * 0.0).backward()
    if gsync is not None:
        gsync.sync()  # an idle rank sends zeros
    torch.save({n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None},
               os.path.join(tmpdir, f"g{rank}.pt"))
    ddp.barrier(info)
    ddp.cleanup()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("B,world,impl", [(6, 4, "sync"), (6, 4, "ddp"), (3, 4, "sync"), (3, 4, "ddp")],
                         ids=["b6w4-sync", "b6w4-ddp", "b3w4-idle-sync", "b3w4-idle-ddp"])
def test_uneven_global_batch_matches_full_batch(B, world, impl):
    """world 4, batch 6 (2,2,1,1) and batch 3 (1,1,1 + an idle rank) reproduce the
    single-process gradient of the whole batch (RAFT-small: no BatchNorm)."""
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss

    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(world, ddp.free_port(), tmp, B, impl), nprocs=world, start_method="spawn")
        grads = [torch.load(os.path.join(tmp, f"g{r}.pt"), weights_only=True) for r in range(world)]
    torch.manual_seed(0)
    model = RAFT(Namespace(small=True, mixed_precision=False))
    i1, i2, flow, valid = _batch(B)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)  # as the workers: the CPU conv backward's sums depend on the thread split
    try:
        loss, _ = sequence_loss(model(i1, i2, iters=2), flow, valid)
        loss.backward()
    finally:
        torch.set_num_threads(nt)
    n_checked = 0
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        for r in range(world):  # every replica holds the same, full-batch gradient
            torch.testing.assert_close(grads[r][n], p.grad, rtol=2e-4, atol=2e-6)
        n_checked += 1
    assert n_checked > 50


def _train_worker(rank, world, port, tmpdir, batch, split):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import train as train_cli
    from raft_ros_amd.train import trainer

    ck = os.path.join(tmpdir, f"ckpt{rank}")
    logs = os.path.join(tmpdir, f"runs{rank}")
    args = train_cli.build_parser().parse_args(
        ["--name", "gb", "--stage", "synthetic", "--small", "--batch_size", str(batch), "--image_size", "128", "128",
         "--num_steps", "2", "--iters", "2", "--num_workers", "0", "--ckpt_dir", ck, "--log_dir", logs,
         "--lr", "4e-4", "--batch_split", split])
    torch.manual_seed(args.seed + rank)  # as train.py's _main: different init per rank
    os.makedirs(ck, exist_ok=True)

    def dump(model, info):
        torch.save({k: v.detach().clone() for k, v in model.state_dict().items()},
                   os.path.join(tmpdir, f"final{rank}.pt"))

    trainer.train(args, on_finish=dump)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("batch,split", [(3, "balanced"), (2, "chunk")])
def test_train_two_ranks_replicas_in_sync_rank0_writes(batch, split):
    """train.py --stage synthetic on 2 gloo ranks for 3 steps (uneven 2 + 1 split, and a batch
    of 2): the replicas end bitwise equal and only rank 0 writes checkpoint files."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_train_worker, args=(2, ddp.free_port(), tmp, batch, split), nprocs=2,
                           start_method="spawn")
        s0 = torch.load(os.path.join(tmp, "final0.pt"), weights_only=True)
        s1 = torch.load(os.path.join(tmp, "final1.pt"), weights_only=True)
        assert sorted(os.listdir(os.path.join(tmp, "ckpt0"))) == ["gb.pth", "gb.state.pt"]
        assert os.listdir(os.path.join(tmp, "ckpt1")) == []
        ck = torch.load(os.path.join(tmp, "ckpt0", "gb.pth"), weights_only=True)
    init = {}
    torch.manual_seed(1234)
    from raft_ros_amd.models import RAFT

    for k, v in RAFT(Namespace(small=True, mixed_precision=False)).state_dict().items():
        init[k] = v
    moved = 0
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
        assert torch.equal(ck["module." + k], s0[k]), k
        moved += int(not torch.equal(s0[k], init[k]))
    assert moved > 50  # the optimizer did update the (rank-0-broadcast) weights


def _bn_train_worker(rank, world, port, tmpdir):
    """RAFT-base, chairs stage (trainable BatchNorm), global batch 1 on 2 ranks: rank 1 is idle."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import train as train_cli
    from raft_ros_amd.data import datasets
    from raft_ros_amd.train import trainer

    ck = os.path.join(tmpdir, f"ckpt{rank}")
    args = train_cli.build_parser().parse_args(
        ["--name", "bn", "--stage", "chairs", "--batch_size", "1", "--image_size", "128", "128",
         "--num_steps", "1", "--iters", "2", "--num_workers", "0", "--ckpt_dir", ck,
         "--log_dir", os.path.join(tmpdir, f"runs{rank}"), "--lr", "4e-4"])
    torch.manual_seed(args.seed + rank)
    os.makedirs(ck, exist_ok=True)

    def fetch(a):  # the chairs stage's BN semantics on synthetic batches (no dataset here)
        b = Namespace(**vars(a))
        b.stage = "synthetic"
        return datasets.fetch_dataloader(b)

    trainer.fetch_dataloader = fetch
    trainer.VAL_FREQ = 2  # a checkpoint + (empty) validation after the second step

    def dump(model, info):
        torch.save({k: v.detach().clone() for k, v in model.state_dict().items()},
                   os.path.join(tmpdir, f"final{rank}.pt"))

    trainer.train(args, on_finish=dump)


@pytest.mark.timeout(900)
def test_idle_rank_bn_statistics_broadcast_before_validation():
    """an idle GradSync rank never runs a forward, so its BatchNorm running
    statistics stay at 0 / 1 and its shard of a sharded validation would be scored with them.
    The trainer broadcasts rank 0's buffers before validating: both ranks end with rank 0's
    (trained, non-initial) statistics."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_bn_train_worker, args=(2, ddp.free_port(), tmp), nprocs=2, start_method="spawn")
        s0 = torch.load(os.path.join(tmp, "final0.pt"), weights_only=True)
        s1 = torch.load(os.path.join(tmp, "final1.pt"), weights_only=True)
    bn = [k for k in s0 if k.startswith("cnet.") and k.endswith("running_mean")]
    assert bn
    assert any(float(s0[k].abs().max()) > 0 for k in bn)  # rank 0 did update them
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k


def _scaler_worker(rank, world, port, tmpdir, init_idle):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from raft_ros_amd.train.trainer import init_idle_scaler

    info = ddp.init_distributed(device_type="cpu")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))
    _, gsync = ddp.data_parallel(model, info, impl="sync")
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    scaler = torch.amp.GradScaler("cpu", init_scale=1024.0, enabled=True)
    err = ""
    for step in range(3):
        opt.zero_grad(set_to_none=True)
        if rank == 0:  # the one busy rank of a global batch of 1
            x = torch.randn(4, 8, generator=torch.Generator().manual_seed(step))
            scaler.scale(model(x).square().mean() * world).backward()
        elif init_idle:
            init_idle_scaler(scaler, torch.device("cpu"))
        gsync.sync()
        try:
            scaler.unscale_(opt)
        except Exception as e:  # noqa: BLE001 -- the failure mode under test
            err = repr(e)
            break
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        scaler.step(opt)
        scaler.update()
    torch.save({"state": model.state_dict(), "err": err, "scale": float(scaler.get_scale())},
               os.path.join(tmpdir, f"s{rank}.pt"))
    if not err:
        ddp.barrier(info)
    ddp.cleanup()


@pytest.mark.timeout(300)
def test_fp16_gradscaler_with_an_idle_rank():
    """with --amp_dtype fp16 the GradScaler is enabled, and a GradSync rank with
    no sample never called scaler.scale(), so unscale_ failed ('_scale is None') while the busy
    ranks waited.  The trainer initialises the idle rank's scaler: both ranks step in lockstep and
    end bitwise equal with the same scale.  Without it, the idle rank's unscale_ raises."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_scaler_worker, args=(2, ddp.free_port(), tmp, True), nprocs=2, start_method="spawn")
        r = [torch.load(os.path.join(tmp, f"s{i}.pt"), weights_only=True) for i in range(2)]
    assert r[0]["err"] == "" and r[1]["err"] == ""
    assert r[0]["scale"] == r[1]["scale"]
    for k in r[0]["state"]:
        assert torch.equal(r[0]["state"][k], r[1]["state"][k]), k
    # negative control, one rank only (no collective for the failing rank to strand)
    sc = torch.amp.GradScaler("cpu", enabled=True)
    lin = torch.nn.Linear(2, 2)
    for p in lin.parameters():
        p.grad = torch.zeros_like(p)
    with pytest.raises(Exception):
        sc.unscale_(torch.optim.AdamW(lin.parameters()))


def _usage_worker(rank, world, port, tmpdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    info = ddp.init_distributed(device_type="cpu")
    a, b = torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)
    model = torch.nn.ModuleList([a, b])
    _, gsync = ddp.data_parallel(model, info, impl="sync")
    x = torch.randn(2, 4)
    a(x).sum().backward()  # step 1: b unused
    gsync.sync()
    out = {"b_none": b.weight.grad is None}
    model.zero_grad(set_to_none=True)
    b(a(x)).sum().backward()  # b joins (every rank): a silent drop before the fix
    try:
        gsync.sync()
        out["raised"] = False
    except RuntimeError:
        out["raised"] = True
    gsync.reset_usage()  # collective re-detection
    gsync.sync()
    out["b_after_reset"] = b.weight.grad is not None
    torch.save(out, os.path.join(tmpdir, f"u{rank}.pt"))
    ddp.barrier(info)
    ddp.cleanup()


@pytest.mark.timeout(300)
def test_gradsync_refuses_to_drop_a_late_gradient():
    """a parameter without a gradient on the first sync was frozen to
    p.grad = None and a later gradient dropped silently; now the sync raises, and
    reset_usage() re-detects the trained set."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_usage_worker, args=(2, ddp.free_port(), tmp), nprocs=2, start_method="spawn")
        for r in range(2):
            out = torch.load(os.path.join(tmp, f"u{r}.pt"), weights_only=True)
            assert out == {"b_none": True, "raised": True, "b_after_reset": True}, out
