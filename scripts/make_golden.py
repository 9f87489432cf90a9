#!/usr/bin/env python3
"""Golden fixtures from the REAL reference implementation (run on CPU, here, once).

For RAFT base and small with seed-0 random-init weights (``torch.manual_seed(0)`` before
constructing the reference ``core.raft.RAFT``; our ``RAFT`` consumes the RNG identically, so
``torch.manual_seed(0); RAFT(args)`` rebuilds the same weights -- verified below and by a
per-tensor checksum stored in the fixture) and the reference's own demo frames
(``demo-frames/frame_0016..0018.png``, 436x1024, read with PIL as demo.py:20-23 does), run the
reference forward exactly as demo.py:56-62 does: InputPadder (sintel mode, 436 -> 440),
``test_mode=True``, 20 iterations, fp32 on the CPU.  Stored per model and frame pair:

* ``flow_low`` (1, 2, 55, 128) fp32, complete;
* ``flow_up`` (1, 2, 440, 1024) fp32 subsampled every 4th row / column (keeps the file small);
* ``ck_<name>``: sum of squares of every parameter (weight checksum).

Output: ``tests/fixtures/golden_demo_frames.npz`` (consumed by tests/test_golden_gpu.py and
tests/test_golden_cpu.py).  The reference is imported read-only (no bytecode written).
"""
from __future__ import annotations

import importlib
import os
import sys
import time
from argparse import Namespace

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = "/root/reference"
FRAMES = ["frame_0016.png", "frame_0017.png", "frame_0018.png"]
ITERS = 20
SUB = 4


def load_frames():
    out = []
    for f in FRAMES:
        img = np.array(Image.open(os.path.join(ROOT, "demo-frames", f))).astype(np.uint8)
        out.append(torch.from_numpy(img).permute(2, 0, 1).float()[None])
    return out


def checksums(model) -> dict:
    return {k: float((v.double() ** 2).sum()) for k, v in model.state_dict().items() if v.dtype.is_floating_point}


def main():
    sys.dont_write_bytecode = True
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.path.append(REFERENCE)
    ref_raft = importlib.import_module("core.raft")
    ref_utils = importlib.import_module("core.utils.utils")
    sys.path.insert(0, ROOT)
    from raft_ros_amd.models import RAFT

    torch.set_num_threads(8)
    frames = load_frames()
    out = {"iters": np.array(ITERS), "sub": np.array(SUB)}
    for name, small in (("base", False), ("small", True)):
        torch.manual_seed(0)
        model = ref_raft.RAFT(Namespace(small=small, mixed_precision=False, alternate_corr=False)).eval()
        torch.manual_seed(0)
        ours = RAFT(Namespace(small=small, mixed_precision=False)).state_dict()
        assert all(torch.equal(ours[k], v) for k, v in model.state_dict().items()), "init parity"
        for k, v in checksums(model).items():
            out[f"{name}/ck/{k}"] = np.array(v)
        for p in range(len(frames) - 1):
            i1, i2 = frames[p], frames[p + 1]
            padder = ref_utils.InputPadder(i1.shape)
            a, b = padder.pad(i1, i2)
            t0 = time.time()
            with torch.no_grad():
                lo, up = model(a, b, iters=ITERS, test_mode=True)
            print(f"{name} pair {p}: {a.shape[-2:]} {time.time() - t0:.1f} s, |flow| mean {up.norm(dim=1).mean():.3f}")
            out[f"{name}/pair{p}/flow_low"] = lo.numpy().astype(np.float32)
            out[f"{name}/pair{p}/flow_up_sub"] = up[:, :, ::SUB, ::SUB].numpy().astype(np.float32).copy()
    path = os.path.join(ROOT, "tests", "fixtures", "golden_demo_frames.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
