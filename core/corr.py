"""Reference core/corr.py names -> raft_ros_amd correlation blocks.

``CorrBlock`` is the all-pairs pyramid (HIP/MFMA on GPU), ``AlternateCorrBlock``
the memory-efficient local correlation (HIP kernel, trainable)."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))

from raft_ros_amd.ops.corr import CorrPyramid as CorrBlock  # noqa: E402,F401
from raft_ros_amd.ops.corr import LocalCorrPyramid as AlternateCorrBlock  # noqa: E402,F401
