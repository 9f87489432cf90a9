"""Native (HIP/CDNA4) ops of raft_ros_amd with their autograd wiring.

``torch.ops.raft_amd.*`` are registered by the in-tree extension
``raft_ros_amd/_C.so`` (built from ``raft_ros_amd/csrc``); the
``reference`` module holds the pure-PyTorch equivalents used on CPU and as the
numerical oracle in tests.
"""
from ._ext import is_loaded, library_path, load_error, use_native  # noqa: F401
from .corr import CorrPyramid, LocalCorrPyramid  # noqa: F401
from .upsample import convex_upsample, upflow8  # noqa: F401
from . import reference  # noqa: F401
