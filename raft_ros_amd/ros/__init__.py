"""ROS1 integration (node, frame pairing, inference wrapper); rospy is optional."""
from .node import FlowInference, FramePairer, RaftRosNode  # noqa: F401
