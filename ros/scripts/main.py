#!/usr/bin/env python3
"""raft_ros inference node: rosrun raft_ros main.py (see ros/launch/run.launch)."""
import os
import sys

sys.path.append(os.path.join(os.path.dirname(os.path.realpath(__file__)), "..", ".."))

from raft_ros_amd.ros.node import main  # noqa: E402

if __name__ == "__main__":
    main()
