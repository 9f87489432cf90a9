#!/usr/bin/env python3
"""Training-gradient golden fixture from the REAL reference implementation (CPU, fp32, once).

One reference training step's gradients (``train.py:172-175``: forward with ``iters``, the
reference's ``sequence_loss`` (``train.py:47-72``, its own source text, parsed out of the
read-only reference file -- ``train.py`` itself cannot be imported here: it needs cv2,
matplotlib and tensorboard), ``loss.backward()``) for RAFT base and small with seed-0 weights
(``torch.manual_seed(0)`` before construction; our ``RAFT`` consumes the RNG identically, see
``scripts/make_golden.py``), in train mode (the base context encoder's BatchNorm on batch
statistics, as the chairs stage trains it), on:

* a batch of two 128x160 crops of the reference's demo frames (``frame_0016`` -> ``0017``,
  at rows / columns (96, 288) and (224, 640));
* a synthetic smooth ground-truth flow and a valid mask with an invalid band;
* 3 refinement iterations, gamma 0.8.

Stored per model: the loss, the last upsampled prediction, and per parameter the gradient
norm plus its projection on 16 fixed Gaussian directions (``projections(name, numel)``,
regenerated bit-identically by the tests from a name-seeded CPU generator), or the full
gradient for tensors of at most 4096 elements.  Output: ``tests/fixtures/golden_grads.npz``
(tests/test_golden_cpu.py, tests/test_golden_gpu.py).
"""
from __future__ import annotations

import ast
import importlib
import os
import sys
import zlib
from argparse import Namespace

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

ITERS = 3
NPROJ = 16
FULL_MAX = 4096
CROPS = [(96, 288), (224, 640)]
H, W = 128, 160


def projections(name: str, numel: int) -> torch.Tensor:
    """(NPROJ, numel) fixed Gaussian directions for parameter ``name`` (CPU, deterministic)."""
    g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
    return torch.randn(NPROJ, numel, generator=g, dtype=torch.float64)


def batch():
    """(image1, image2, flow_gt, valid): two crops of the demo frames, synthetic smooth GT."""
    from golden import frames

    fr = frames()
    i1 = torch.cat([fr[0][:, :, y:y + H, x:x + W] for y, x in CROPS])
    i2 = torch.cat([fr[1][:, :, y:y + H, x:x + W] for y, x in CROPS])
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                            indexing="ij")
    u = 3.0 * torch.sin(2 * np.pi * xx / W) + 0.02 * yy
    v = 2.0 * torch.cos(2 * np.pi * yy / H) - 0.01 * xx
    flow = torch.stack([torch.stack([u, v]), torch.stack([-v, u + 1.0])])
    valid = torch.ones(2, H, W)
    valid[:, 40:52, :] = 0.0
    valid[1, :, 100:110] = 0.0
    return i1.contiguous(), i2.contiguous(), flow.contiguous(), valid


def reference_sequence_loss():
    """The reference's own ``sequence_loss`` (train.py:47-72), compiled from its source text."""
    src = open(os.path.join(REFERENCE, "train.py")).read()
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "sequence_loss")
    ns = {"torch": torch, "MAX_FLOW": 400}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "reference/train.py", "exec"), ns)
    return ns["sequence_loss"]


def main():
    sys.dont_write_bytecode = True
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.path.append(REFERENCE)
    ref_raft = importlib.import_module("core.raft")
    from raft_ros_amd.models import RAFT

    torch.set_num_threads(8)
    seq_loss = reference_sequence_loss()
    i1, i2, flow, valid = batch()
    out = {"iters": np.array(ITERS), "nproj": np.array(NPROJ), "full_max": np.array(FULL_MAX)}
    for name, small in (("base", False), ("small", True)):
        torch.manual_seed(0)
        model = ref_raft.RAFT(Namespace(small=small, mixed_precision=False, alternate_corr=False))
        torch.manual_seed(0)
        ours = RAFT(Namespace(small=small, mixed_precision=False)).state_dict()
        assert all(torch.equal(ours[k], v) for k, v in model.state_dict().items()), "init parity"
        model.train()
        preds = model(i1, i2, iters=ITERS)
        loss, metrics = seq_loss(preds, flow, valid, 0.8)
        loss.backward()
        out[f"{name}/loss"] = np.array(float(loss))
        out[f"{name}/pred_last"] = preds[-1].detach().numpy().astype(np.float32)
        for pn, p in model.named_parameters():
            g = p.grad.detach().double().reshape(-1)
            out[f"{name}/gnorm/{pn}"] = np.array(float(g.norm()))
            if g.numel() <= FULL_MAX:
                out[f"{name}/gfull/{pn}"] = g.numpy().astype(np.float64)
            else:
                out[f"{name}/gproj/{pn}"] = (projections(pn, g.numel()) @ g).numpy()
        print(f"{name}: loss {float(loss):.6f} epe {metrics['epe']:.4f}, {len(list(model.parameters()))} parameters")
    path = os.path.join(ROOT, "tests", "fixtures", "golden_grads.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
