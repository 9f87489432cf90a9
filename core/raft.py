"""``from core.raft import RAFT`` (reference core/raft.py) -> raft_ros_amd.models.RAFT."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))

from raft_ros_amd.models.raft import RAFT  # noqa: E402,F401
