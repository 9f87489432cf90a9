"""Compatibility package mirroring the reference's ``core/`` layout.

The reference's scripts and its ROS node import ``core.raft.RAFT`` /
``core.utils.flow_viz`` / ``core.utils.utils.InputPadder`` (or, after
``sys.path.append('core')``, ``raft``, ``datasets``, ``utils.*``).  These thin
modules re-export the MI355X implementation from ``raft_ros_amd`` so code
written against the reference keeps working unchanged.
"""
import os as _os
import sys as _sys

_root = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _root not in _sys.path:
    _sys.path.append(_root)
