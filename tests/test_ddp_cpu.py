"""Distributed data parallel on CPU (gloo, 2 processes): DDP with the per-rank share of
the batch must reproduce the single-process gradient of the full batch."""
import os
import tempfile
from argparse import Namespace

import pytest
import torch
import torch.multiprocessing as mp

from raft_ros_amd.parallel import ddp


def _worker(rank, world, port, tmpdir, bf16=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss

    info = ddp.init_distributed(device_type="cpu")
    torch.manual_seed(0)
    model = RAFT(Namespace(small=True, mixed_precision=False))
    net = ddp.wrap_model(model, info, bf16_grads=bf16)
    i1, i2, flow, valid = synthetic_batch(4, 128, 128, max_disp=4, seed=7)
    sl = slice(2 * rank, 2 * rank + 2)
    loss, metrics = sequence_loss(net(i1[sl], i2[sl], iters=2), flow[sl], valid[sl])
    loss.backward()
    red = ddp.all_reduce_mean({"loss": loss.item(), "rank": float(rank)}, info)
    if rank == 0:
        torch.save({n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None},
                   os.path.join(tmpdir, "ddp.pt"))
        torch.save(red, os.path.join(tmpdir, "red.pt"))
    ddp.barrier(info)
    ddp.cleanup()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("bf16", [False, True], ids=["fp32", "bf16_hook"])
def test_ddp_gradients_match_full_batch(bf16):
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss

    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, ddp.free_port(), tmp, bf16), nprocs=2, start_method="spawn")
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
