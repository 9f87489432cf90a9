"""Reference core/utils/utils.py names -> raft_ros_amd.utils.utils."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))

from raft_ros_amd.utils.utils import (InputPadder, bilinear_sampler, coords_grid, forward_interpolate,  # noqa: E402,F401
                                      upflow8)
