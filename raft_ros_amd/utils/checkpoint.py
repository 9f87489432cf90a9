"""Checkpoint I/O compatible with the reference ``raft-*.pth`` files.

The reference saves ``nn.DataParallel(RAFT).state_dict()`` -- every key is
prefixed ``module.`` (train.py:187,212) -- and every loader wraps the model in
DataParallel only to strip that prefix again (demo.py:43-46, evaluate.py:
178-179, ros/scripts/main.py:54-56), with no ``map_location`` (so a
GPU-saved file fails on CPU-only hosts).  Here:

* ``save_weights`` writes exactly that format (OrderedDict, ``module.`` keys),
  so the files are interchangeable with the reference's;
* ``load_weights`` accepts prefixed or plain state dicts, maps to any device,
  and loads with ``torch.load(weights_only=True)`` (no unpickling of code);
* ``save_state`` / ``load_state`` add a resume sidecar (optimizer, scheduler,
  scaler, step, RNG states) so ``--restore_ckpt`` can resume exactly, which the
  reference cannot (checkpoint row).
"""
from __future__ import annotations

import os
import random
from collections import OrderedDict
from typing import Optional

import numpy as np
import torch

PREFIX = "module."


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


def strip_prefix(sd):
    if any(k.startswith(PREFIX) for k in sd):
        return OrderedDict((k[len(PREFIX):] if k.startswith(PREFIX) else k, v) for k, v in sd.items())
    return OrderedDict(sd)


def save_weights(model, path: str) -> None:
    """Save in the reference's DataParallel format (``module.``-prefixed keys)."""
    sd = _unwrap(model).state_dict()
    out = OrderedDict((PREFIX + k, v.detach().cpu()) for k, v in sd.items())
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(out, tmp)
    os.replace(tmp, path)


def load_weights(model, path: str, strict: bool = True, map_location="cpu"):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    return _unwrap(model).load_state_dict(strip_prefix(sd), strict=strict)


def state_path(weights_path: str) -> str:
    root, _ = os.path.splitext(weights_path)
    return root + ".state.pt"


def _py_rng_state():
    """``random.getstate()`` as tensors/ints only, so ``torch.load(weights_only=True)`` can read it."""
    version, internal, gauss = random.getstate()
    return {"version": int(version), "internal": torch.tensor(internal, dtype=torch.int64),
            "gauss": None if gauss is None else float(gauss)}


def _set_py_rng_state(st) -> None:
    if not isinstance(st, dict):  # older sidecars stored an unusable repr string
        return
    random.setstate((st["version"], tuple(int(x) for x in st["internal"].tolist()), st["gauss"]))


def save_state(path: str, optimizer, scheduler, scaler, step: int) -> None:
    np_state = np.random.get_state()
    state = {
        "optimizer": optimizer.state_dict(),
        "scheduler": scheduler.state_dict() if scheduler is not None else None,
        "scaler": scaler.state_dict() if scaler is not None else None,
        "step": int(step),
        "torch_rng": torch.get_rng_state(),
        "cuda_rng": torch.cuda.get_rng_state_all() if torch.cuda.is_available() else [],
        "numpy_rng": {"name": np_state[0], "keys": torch.from_numpy(np_state[1].astype(np.int64)),
                      "pos": int(np_state[2]), "has_gauss": int(np_state[3]), "cached": float(np_state[4])},
        "python_rng": _py_rng_state(),
    }
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_state(path: str, optimizer, scheduler, scaler, map_location="cpu") -> Optional[int]:
    if not os.path.exists(path):
        return None
    st = torch.load(path, map_location=map_location, weights_only=True)
    optimizer.load_state_dict(st["optimizer"])
    if scheduler is not None and st.get("scheduler") is not None:
        scheduler.load_state_dict(st["scheduler"])
    if scaler is not None and st.get("scaler") is not None:
        scaler.load_state_dict(st["scaler"])
    torch.set_rng_state(st["torch_rng"])
    if torch.cuda.is_available() and st.get("cuda_rng"):
        torch.cuda.set_rng_state_all(st["cuda_rng"])
    n = st.get("numpy_rng")
    if n:
        np.random.set_state((n["name"], n["keys"].numpy().astype(np.uint32), n["pos"], n["has_gauss"], n["cached"]))
    _set_py_rng_state(st.get("python_rng"))
    return int(st["step"])
