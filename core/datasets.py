"""Reference core/datasets.py names -> raft_ros_amd.data.datasets."""
import os as _os
import sys as _sys

_sys.path.append(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))

from raft_ros_amd.data.datasets import (HD1K, KITTI, FlowDataset, FlyingChairs, FlyingThings3D,  # noqa: E402,F401
                                        MpiSintel, fetch_dataloader)
