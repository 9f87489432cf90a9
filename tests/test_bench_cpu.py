"""bench.py launch contract on CPU (gloo): ``--gpus N`` without torchrun spawns N ranks
itself and reports the real world size; the JSON line carries every required key."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "allreduce_ms"}


def _bench(*extra, env=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--small", "--image_size", "128",
           "128", "--batch", "1", "--steps", "1", "--warmup", "0", "--iters", "2", *extra]
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=500, cwd=ROOT, env=e)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_bench_spawns_ranks_for_gpus_flag():
    r = _bench("--gpus", "2")
    assert KEYS <= set(r), set(KEYS) - set(r)
    assert r["n_gpus"] == 2
    assert r["config"]["parallelism"] == "dp2"
    assert r["config"]["dp_impl"] == "sync"  # GradSync (parallel/grad_sync.py)
    assert r["config"]["global_batch"] == 2
    assert r["allreduce_ms"] > 0


@pytest.mark.timeout(600)
def test_bench_single_process_default():
    r = _bench()
    assert r["n_gpus"] == 1 and r["allreduce_ms"] == 0.0
    assert r["steps"] == 1 and r["warmup"] == 0


@pytest.mark.timeout(600)
def test_bench_under_torchrun_driver_launch():
    """The driver's multi-GPU launch: python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N (here gloo on
    the CPU, N = 2): one JSON line from rank 0 with the world size and the global batch."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--small", "--image_size", "128", "128", "--batch", "1", "--steps", "1", "--warmup", "0", "--iters", "2"]
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=500, cwd=ROOT, env=e)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 2
    assert r["scaling"] == "weak" and r["allreduce_ms"] > 0


@pytest.mark.timeout(600)
def test_bench_global_batch_strong_scaling_with_idle_rank():
    """--global_batch: the trainer's global-batch split (train_standard.sh on 8 GPUs runs batch 6
    as 1,1,1,1,1,1,0,0); here 1 pair over 2 ranks leaves rank 1 idle -- it still joins the
    gradient all-reduce and the optimizer step, and the job reports strong scaling."""
    r = _bench("--gpus", "2", "--global_batch", "1", "--steps", "2")
    assert r["scaling"] == "strong" and r["n_gpus"] == 2
    assert r["config"]["global_batch"] == 1 and r["config"]["rank_batches"] == [1, 0]
    assert r["vs_baseline"] is None
    assert abs(r["value"] - 1 * 2 / (r["ms_per_step"] * 2 / 1000.0)) / r["value"] < 1e-2
