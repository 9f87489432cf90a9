"""Loader for the in-tree native extension ``raft_ros_amd/_C.so``.

The extension registers its ops in the ``torch.ops.raft_amd`` namespace
(see ``raft_ros_amd/csrc/bindings.cpp``).  On a machine with a GPU the HIP
path is mandatory: if the library is missing or fails to load, GPU callers get
a loud error instead of a silent PyTorch fallback.  Set
``RAFT_AMD_ALLOW_TORCH_FALLBACK=1`` to opt into the pure-PyTorch reference
ops on a GPU anyway (debugging only).
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

_LIB_PATH = Path(__file__).resolve().parent.parent / "_C.so"
_loaded = False
_load_error: str | None = None


def _try_load() -> bool:
    global _loaded, _load_error
    if _loaded:
        return True
    if _load_error is not None:
        return False
    if not _LIB_PATH.exists():
        _load_error = f"{_LIB_PATH} not built (run `python -m raft_ros_amd.csrc.build`)"
        return False
    try:
        torch.ops.load_library(str(_LIB_PATH))
        _loaded = True
    except Exception as exc:  # pragma: no cover - depends on the host
        _load_error = f"failed to load {_LIB_PATH}: {exc}"
    if _loaded:
        from . import _meta

        _meta.register()  # FakeTensor / meta-device shape functions of every op
    return _loaded


def library_path() -> Path:
    return _LIB_PATH


def is_loaded() -> bool:
    return _try_load()


def load_error() -> str | None:
    _try_load()
    return _load_error


def fallback_allowed() -> bool:
    return os.environ.get("RAFT_AMD_ALLOW_TORCH_FALLBACK", "0") == "1"


_backend = "native"


def set_backend(name: str) -> None:
    """'native' (default: HIP kernels on GPU) or 'reference' (the reference's
    PyTorch op sequence, used only to measure the eager baseline)."""
    global _backend
    if name not in ("native", "reference"):
        raise ValueError(name)
    _backend = name


def get_backend() -> str:
    return _backend


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU and the native op must be used.

    Raises if the tensor is on the GPU but the HIP extension is unavailable
    (unless the torch fallback was explicitly allowed).
    """
    if not t.is_cuda or _backend == "reference":
        return False
    if _try_load():
        return True
    if fallback_allowed():
        return False
    raise RuntimeError(
        "raft_ros_amd native HIP extension is required on the GPU but is unavailable: "
        f"{_load_error}. Build it with `python -m raft_ros_amd.csrc.build` "
        "(or set RAFT_AMD_ALLOW_TORCH_FALLBACK=1 to debug with the PyTorch reference ops)."
    )


def ops():
    if not _try_load():
        raise RuntimeError(f"raft_ros_amd native extension unavailable: {_load_error}")
    return torch.ops.raft_amd
