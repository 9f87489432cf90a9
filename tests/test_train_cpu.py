"""Loss, optimizer schedule, checkpoints and a short CPU training run."""
import json
import os
from argparse import Namespace

import torch

from raft_ros_amd.models import RAFT
from raft_ros_amd.train.loss import metrics_to_host, sequence_loss
from raft_ros_amd.train.optim import fetch_optimizer
from raft_ros_amd.utils import checkpoint


def _reference_sequence_loss(preds, gt, valid, gamma=0.8, max_flow=400):
    """The reference formula (train.py:47-72), written out for comparison."""
    n = len(preds)
    mag = torch.sum(gt ** 2, dim=1).sqrt()
    valid = (valid >= 0.5) & (mag < max_flow)
    loss = 0.0
    for i in range(n):
        loss += gamma ** (n - i - 1) * (valid[:, None] * (preds[i] - gt).abs()).mean()
    epe = torch.sum((preds[-1] - gt) ** 2, dim=1).sqrt().view(-1)[valid.view(-1)]
    return loss, {"epe": epe.mean().item(), "1px": (epe < 1).float().mean().item(),
                  "3px": (epe < 3).float().mean().item(), "5px": (epe < 5).float().mean().item()}


def test_sequence_loss_matches_reference_formula():
    torch.manual_seed(0)
    gt = torch.randn(2, 2, 16, 20) * 5
    gt[0, :, 0, 0] = 1000  # |gt| >= 400 -> excluded
    valid = (torch.rand(2, 16, 20) > 0.2).float()
    preds = [gt + torch.randn_like(gt) * s for s in (3.0, 2.0, 1.0)]
    loss, m = sequence_loss(preds, gt, valid, gamma=0.85)
    rl, rm = _reference_sequence_loss(preds, gt, valid, gamma=0.85)
    torch.testing.assert_close(loss, torch.as_tensor(rl, dtype=loss.dtype))
    mh = metrics_to_host(m)
    for k in rm:
        assert abs(mh[k] - rm[k]) < 1e-5, k


def test_onecycle_schedule():
    model = torch.nn.Linear(2, 2)
    args = Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000)
    opt, sched = fetch_optimizer(args, model)
    lrs = []
    for _ in range(1100):
        lrs.append(sched.get_last_lr()[0])
        opt.step()
        sched.step()
    peak = max(range(len(lrs)), key=lambda i: lrs[i])
    assert abs(peak - int(0.05 * 1100)) <= 2 and abs(max(lrs) - 4e-4) < 1e-9
    assert lrs[-1] < 1e-6


def test_checkpoint_format_and_roundtrip(tmp_path):
    m = RAFT(Namespace(small=True, mixed_precision=False))
    p = str(tmp_path / "ckpt" / "raft.pth")
    checkpoint.save_weights(m, p)
    sd = torch.load(p, weights_only=True)
    assert all(k.startswith("module.") for k in sd) and len(sd) == 106
    m2 = RAFT(Namespace(small=True, mixed_precision=False))
    checkpoint.load_weights(m2, p)
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    # plain (un-prefixed) state dicts load too
    torch.save(m.state_dict(), str(tmp_path / "plain.pth"))
    checkpoint.load_weights(m2, str(tmp_path / "plain.pth"))


def test_resume_state_roundtrip(tmp_path):
    model = torch.nn.Linear(3, 3)
    args = Namespace(lr=1e-3, wdecay=1e-4, epsilon=1e-8, num_steps=100)
    opt, sched = fetch_optimizer(args, model)
    for _ in range(5):
        model(torch.randn(4, 3)).sum().backward()
        opt.step()
        sched.step()
    p = str(tmp_path / "s.state.pt")
    checkpoint.save_state(p, opt, sched, None, 5)
    expect = torch.rand(3)
    opt2, sched2 = fetch_optimizer(args, model)
    assert checkpoint.load_state(p, opt2, sched2, None) == 5
    assert sched2.get_last_lr() == sched.get_last_lr()
    torch.manual_seed(0)


def test_train_cli_runs_on_cpu(tmp_path, monkeypatch):
    import train

    monkeypatch.chdir(tmp_path)
    path = train.main(["--name", "t", "--stage", "synthetic", "--small", "--num_steps", "3", "--batch_size", "2",
                       "--image_size", "128", "128", "--iters", "2", "--gpus", "0", "--num_workers", "0",
                       "--lr", "1e-4"])
    assert os.path.exists(path) and os.path.exists(checkpoint.state_path(path))
    sd = torch.load(path, weights_only=True)
    assert all(k.startswith("module.") for k in sd)
    # resume continues from the saved step
    path2 = train.main(["--name", "t2", "--stage", "synthetic", "--small", "--num_steps", "5", "--batch_size", "2",
                        "--image_size", "128", "128", "--iters", "2", "--gpus", "0", "--num_workers", "0",
                        "--restore_ckpt", path, "--resume"])
    assert os.path.exists(path2)
    assert os.path.exists(os.path.join("runs", "t", "metrics.jsonl"))


def test_resume_restores_python_and_numpy_rng(tmp_path):
    import random

    import numpy as np

    m = RAFT(Namespace(small=True))
    opt, sch = fetch_optimizer(Namespace(lr=1e-4, wdecay=1e-5, epsilon=1e-8, num_steps=10), m)
    random.seed(123)
    np.random.seed(321)
    p = str(tmp_path / "s.state.pt")
    checkpoint.save_state(p, opt, sch, None, 5)
    expect = (random.random(), float(np.random.rand()))
    random.seed(999)
    np.random.seed(999)
    assert checkpoint.load_state(p, opt, sch, None) == 5
    assert (random.random(), float(np.random.rand())) == expect


def test_logger_reduces_metrics_before_printing(tmp_path, capsys):
    from raft_ros_amd.train.logger import Logger

    calls = []

    def reduce_fn(m):
        calls.append(dict(m))
        return {k: 2 * v for k, v in m.items()}

    lg = Logger(log_dir=str(tmp_path), sum_freq=2, reduce_fn=reduce_fn)
    lg.push({"epe": torch.tensor(1.0)})
    out = capsys.readouterr().out
    assert calls == [{"epe": 0.5}] and "1.0000" in out  # window of 2 -> mean 0.5, reduced x2
    lg.close()
