"""Reference core/utils/flow_viz.py names -> raft_ros_amd.utils.flow_viz."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))

from raft_ros_amd.utils.flow_viz import flow_to_image, flow_uv_to_colors, make_colorwheel  # noqa: E402,F401
