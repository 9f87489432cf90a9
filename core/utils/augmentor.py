"""Reference core/utils/augmentor.py names -> raft_ros_amd.data.augmentor."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))

from raft_ros_amd.data.augmentor import ColorJitter, FlowAugmentor, SparseFlowAugmentor  # noqa: E402,F401
