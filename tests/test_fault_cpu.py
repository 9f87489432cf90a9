"""Failure detection: injected faults end a multi-rank job cleanly
instead of hanging it, and a non-finite step is skipped on every rank.

The multi-rank cases run the real ``train.py`` under ``torch.distributed.run`` with two
gloo ranks on the CPU (RAFT-small, synthetic stage, 128x128)."""
import os
import subprocess
import sys
import time

import pytest

from raft_ros_amd.parallel import ddp
from raft_ros_amd.utils import fault

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_fault_spec():
    f = fault.parse("rank=1,step=2,kind=exit,code=9")
    assert (f.kind, f.step, f.rank, f.code) == ("exit", 2, 1, 9)
    assert f.hits(2, 1) and not f.hits(2, 0) and not f.hits(1, 1)
    g = fault.parse("kind=nan")
    assert g.rank is None and g.step == 0 and g.hits(0, 5)
    for bad in ("kind=boom", "rank=1", "kind=exit,colour=red", "kind"):
        with pytest.raises(ValueError):
            fault.parse(bad)


def test_injector_is_inert_without_env(monkeypatch):
    import torch

    monkeypatch.delenv(fault.ENV, raising=False)
    inj = fault.Injector.from_env(0)
    inj.before_step(0)
    x = torch.ones(())
    assert inj.on_loss(0, x) is x


def _torchrun(tmp_path, spec, extra_env=None, steps=4, timeout=240):
    env = dict(os.environ, **{fault.ENV: spec, "OMP_NUM_THREADS": "2", "PYTHONPATH": ROOT})
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(ddp.free_port()),
           os.path.join(ROOT, "train.py"), "--name", "f", "--stage", "synthetic", "--small",
           "--num_steps", str(steps), "--batch_size", "2", "--image_size", "128", "128", "--iters", "2",
           "--num_workers", "0", "--lr", "1e-4", "--ckpt_dir", str(tmp_path / "ck"),
           "--log_dir", str(tmp_path / "runs")]
    t0 = time.monotonic()
    p = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=timeout)
    return p, time.monotonic() - t0


@pytest.mark.parametrize("kind", ["exit", "raise"])
def test_dead_rank_aborts_job(tmp_path, kind):
    """Rank 1 dies (hard exit / exception) at step 1: the launcher must end the whole job
    with a failure status, no final checkpoint written, and no hang."""
    p, dt = _torchrun(tmp_path, f"rank=1,step=1,kind={kind}")
    out = p.stdout + p.stderr
    assert p.returncode != 0, out[-3000:]
    assert ("[fault] rank 1" in out) or ("InjectedFault" in out), out[-3000:]
    assert not (tmp_path / "ck" / "f.pth").exists()
    assert dt < 200


def test_stuck_rank_hits_collective_timeout(tmp_path):
    """Rank 1 stalls before step 1; rank 0 blocks in the gradient all-reduce and must fail
    after RAFT_DIST_TIMEOUT seconds instead of waiting for the stalled peer forever."""
    p, dt = _torchrun(tmp_path, "rank=1,step=1,kind=hang,secs=600", {"RAFT_DIST_TIMEOUT": "8"})
    out = p.stdout + p.stderr
    assert p.returncode != 0, out[-3000:]
    assert "[fault] rank 1: hanging" in out, out[-3000:]
    assert dt < 200  # far below the 600 s stall


def test_nan_step_is_skipped_everywhere(tmp_path, monkeypatch, capsys):
    import train

    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv(fault.ENV, "step=1,kind=nan")
    train.main(["--name", "n", "--stage", "synthetic", "--small", "--num_steps", "2", "--batch_size", "2",
                "--image_size", "128", "128", "--iters", "2", "--gpus", "0", "--num_workers", "0", "--lr", "1e-4"])
    assert "1 non-finite steps skipped" in capsys.readouterr().out
