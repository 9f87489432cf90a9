"""Reference core/update.py names -> raft_ros_amd.models.update."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))

from raft_ros_amd.models.update import (BasicMotionEncoder, BasicUpdateBlock, ConvGRU, FlowHead,  # noqa: E402,F401
                                        SepConvGRU, SmallMotionEncoder, SmallUpdateBlock)
