"""demo.py / evaluate.py command lines on CPU (RAFT-small, synthetic frames)."""
import os

import numpy as np
import torch
from PIL import Image

from raft_ros_amd.data.synthetic import synthetic_batch
from raft_ros_amd.models import RAFT
from raft_ros_amd.utils import checkpoint


def _frames(tmp, n=3, h=128, w=160):
    i1, i2, _, _ = synthetic_batch(1, h, w, seed=5)
    paths = []
    for k, im in enumerate([i1, i2, i1][:n]):
        p = os.path.join(tmp, f"frame_{k:04d}.png")
        Image.fromarray(im[0].permute(1, 2, 0).byte().numpy()).save(p)
        paths.append(p)
    return paths


def test_demo_cli_writes_visualisations(tmp_path):
    import demo
    from argparse import Namespace

    os.makedirs(tmp_path / "frames")
    _frames(str(tmp_path / "frames"), 3)
    model = RAFT(Namespace(small=True, mixed_precision=False))
    ck = str(tmp_path / "m.pth")
    checkpoint.save_weights(model, ck)
    outs = demo.main(["--model", ck, "--small", "--path", str(tmp_path / "frames"), "--device", "cpu",
                      "--iters", "2", "--output", str(tmp_path / "out")])
    assert len(outs) == 2
    vis = np.array(Image.open(outs[0]))
    assert vis.shape == (256, 160, 3)  # [image; flow] stacked


def test_evaluate_cli_synthetic(tmp_path):
    import evaluate
    from argparse import Namespace

    model = RAFT(Namespace(small=True, mixed_precision=False))
    ck = str(tmp_path / "m.pth")
    checkpoint.save_weights(model, ck)
    import raft_ros_amd.eval.validate as V

    res = V.validate_synthetic(model.eval(), iters=2, n_pairs=2, size=(128, 128))
    assert set(res) == {"synthetic-epe", "synthetic-1px", "synthetic-3px", "synthetic-5px"}
    out = evaluate.main(["--model", ck, "--small", "--dataset", "synthetic", "--device", "cpu", "--iters", "1"])
    assert out["synthetic-epe"] >= 0


def test_demo_synthesises_frames_when_path_is_empty(tmp_path, monkeypatch):
    import demo
    from raft_ros_amd.data import synthetic

    # small frames keep the CPU run short; the default sequence is Sintel-sized (436x1024)
    monkeypatch.setattr(synthetic, "demo_sequence",
                        lambda n=6: [f[:, :128, :160] for f in synthetic.__dict__["_demo_full"](3)])
    outs = demo.main(["--small", "--path", str(tmp_path / "frames"), "--device", "cpu", "--iters", "1",
                      "--output", str(tmp_path / "out")])
    assert len(outs) == 2 and len(os.listdir(tmp_path / "frames")) == 3


def test_demo_sequence_shape_and_motion():
    import torch
    from raft_ros_amd.data.synthetic import demo_sequence

    fr = demo_sequence(3, 96, 128)
    assert len(fr) == 3 and fr[0].shape == (3, 96, 128) and fr[0].dtype == torch.uint8
    assert (fr[0].float() - fr[1].float()).abs().mean() > 1.0  # frames actually move


def test_train_refuses_gpu_ids_the_node_does_not_have(monkeypatch):
    """Reference default --gpus 0 1 on a 1-GPU node: a clear error, not a dead rank on cuda:1."""
    import pytest

    import train

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit, match="1 visible GPU"):
        train.check_gpus([0, 1], ndev=1)
    with pytest.raises(SystemExit):
        train.check_gpus([0, 0], ndev=2)
    train.check_gpus([0, 1], ndev=2)
    train.check_gpus([0, 1], ndev=0)  # CPU-only host: not checked
    monkeypatch.setenv("WORLD_SIZE", "2")
    train.check_gpus([0, 1], ndev=1)  # torchrun decides the ranks
