"""Distributed data parallel on CPU (gloo, 2 processes): DDP with the per-rank share of
the batch must reproduce the single-process gradient of the full batch."""
import os
import tempfile
from argparse import Namespace

import pytest
import torch
import torch.multiprocessing as mp

from raft_ros_amd.parallel import ddp


def _worker(rank, world, port, tmpdir, bf16=False, impl="ddp"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss

    info = ddp.init_distributed(device_type="cpu")
    torch.manual_seed(0)
    model = RAFT(Namespace(small=True, mixed_precision=False))
    net, gsync = ddp.data_parallel(model, info, impl=impl, bf16_grads=bf16)
    i1, i2, flow, valid = synthetic_batch(4, 128, 128, max_disp=4, seed=7)
    sl = slice(2 * rank, 2 * rank + 2)
    loss, metrics = sequence_loss(net(i1[sl], i2[sl], iters=2), flow[sl], valid[sl])
    loss.backward()
    if gsync is not None:
        gsync.sync()
    red = ddp.all_reduce_mean({"loss": loss.item(), "rank": float(rank)}, info)
    if rank == 0:
        torch.save({n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None},
                   os.path.join(tmpdir, "ddp.pt"))
        torch.save(red, os.path.join(tmpdir, "red.pt"))
    ddp.barrier(info)
    ddp.cleanup()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("impl", ["ddp", "sync"])
@pytest.mark.parametrize("bf16", [False, True], ids=["fp32", "bf16_hook"])
def test_ddp_gradients_match_full_batch(bf16, impl):
    """DDP (bucketed hooks) and GradSync (one packed all-reduce after the backward, the
    default of train.py) both reproduce the full-batch gradient."""
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss

    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, ddp.free_port(), tmp, bf16, impl), nprocs=2, start_method="spawn")
        grads = torch.load(os.path.join(tmp, "ddp.pt"), weights_only=True)
        red = torch.load(os.path.join(tmp, "red.pt"), weights_only=True)
    assert red["rank"] == 0.5
    torch.manual_seed(0)
    model = RAFT(Namespace(small=True, mixed_precision=False))
    i1, i2, flow, valid = synthetic_batch(4, 128, 128, max_disp=4, seed=7)
    # mean over the two halves == DDP's averaged gradient (no BatchNorm in RAFT-small)
    total = 0
    for sl in (slice(0, 2), slice(2, 4)):
        loss, _ = sequence_loss(model(i1[sl], i2[sl], iters=2), flow[sl], valid[sl])
        total = total + loss / 2
    total.backward()
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        if bf16:  # each rank's contribution is rounded to bf16 before the sum
            # (biases in front of InstanceNorm have a ~0 true gradient: bound those absolutely)
            scale = max(float(q.grad.norm()) for q in model.parameters() if q.grad is not None)
            err = float((grads[n] - p.grad).norm())
            assert err < 1e-2 * max(float(p.grad.norm()), 1e-3 * scale), (n, err, float(p.grad.norm()))
        else:
            torch.testing.assert_close(grads[n], p.grad, rtol=1e-4, atol=1e-6)


def _sync_worker(rank, world, port, tmpdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    info = ddp.init_distributed(device_type="cpu")
    torch.manual_seed(rank)  # different init per rank: GradSync broadcasts rank 0's weights
    m = torch.nn.Sequential(torch.nn.Conv2d(4, 8, 3, padding=1), torch.nn.Conv2d(8, 2, 1),
                            torch.nn.Linear(5, 5))  # the Linear gets no gradient
    m = m.to(memory_format=torch.channels_last)
    _, gsync = ddp.data_parallel(m, info, impl="sync")
    x = torch.randn(2, 4, 6, 6, generator=torch.Generator().manual_seed(10 + rank))
    m[1](m[0](x)).square().mean().backward()
    assert m[0].weight.grad.is_contiguous(memory_format=torch.channels_last)
    gsync.sync()
    torch.save({"w": [p.detach().clone() for p in m.parameters()],
                "g": [None if p.grad is None else p.grad.clone() for p in m.parameters()],
                "strides": [p.grad is None or p.grad.stride() == p.stride() for p in m.parameters()]},
               os.path.join(tmpdir, f"r{rank}.pt"))
    ddp.barrier(info)
    ddp.cleanup()


@pytest.mark.timeout(300)
def test_grad_sync_channels_last_and_missing_grads():
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_sync_worker, args=(2, ddp.free_port(), tmp), nprocs=2, start_method="spawn")
        r = [torch.load(os.path.join(tmp, f"r{k}.pt"), weights_only=True) for k in range(2)]
    for a, b in zip(r[0]["w"], r[1]["w"]):  # rank 0's weights everywhere
        assert torch.equal(a, b)
    assert all(r[0]["strides"]) and all(r[1]["strides"])  # grads keep the parameters' layout
    # recompute both ranks' gradients from rank 0's weights: the synced grad is their mean
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Conv2d(4, 8, 3, padding=1), torch.nn.Conv2d(8, 2, 1), torch.nn.Linear(5, 5))
    with torch.no_grad():
        for p, w in zip(m.parameters(), r[0]["w"]):
            p.copy_(w)
    gs = []
    for rank in range(2):
        m.zero_grad()
        x = torch.randn(2, 4, 6, 6, generator=torch.Generator().manual_seed(10 + rank))
        m[1](m[0](x)).square().mean().backward()
        gs.append([p.grad.clone() if p.grad is not None else torch.zeros_like(p) for p in m.parameters()])
    for i, (g0, g1) in enumerate(zip(*gs)):
        if r[0]["g"][i] is None:  # no rank had a gradient (the Linear): stays None, as in DDP
            assert r[1]["g"][i] is None and i >= 4
            continue
        torch.testing.assert_close(r[0]["g"][i], (g0 + g1) / 2, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(r[1]["g"][i], r[0]["g"][i], rtol=0, atol=0)
