"""Reference core/utils/augmentor.py names -> raft_ros_amd.data.augment."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))

from raft_ros_amd.data.augment import FlowAugmentor, SparseFlowAugmentor  # noqa: E402,F401
