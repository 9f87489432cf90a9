"""Reference core/extractor.py names -> raft_ros_amd.models.extractor."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))

from raft_ros_amd.models.extractor import BasicEncoder, BottleneckBlock, ResidualBlock, SmallEncoder  # noqa: E402,F401
