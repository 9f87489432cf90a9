"""Reference core/utils/frame_utils.py names -> raft_ros_amd.data.frame_utils."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))

from raft_ros_amd.data.frame_utils import (TAG_CHAR, read_gen, readDispKITTI, readFlow, readFlowKITTI,  # noqa: E402,F401
                                           readPFM, writeFlow, writeFlowKITTI, writePFM)
