"""ROS1 optical-flow node (reference ros/scripts/main.py:25-160).

Topics / parameters are those of the reference so existing launch files work:

* subscribes ``rosparam /ROS/prev_img`` and ``/ROS/curr_img`` (sensor_msgs/Image);
* publishes the colour-coded flow on ``/raft_result`` (queue_size 100), encoding
  ``passthrough`` (BGR uint8), header = the *current* image's header with
  ``frame_id = "raft_image"``;
* ``/RAFT/weight_path``, ``/RAFT/is_small``, ``/RAFT/device``; 20 refinement
  iterations, fp32 (``mixed_precision = False``) unless ``/RAFT/mixed_precision``.

Pairing rule (reference :87-114): take the oldest current frame, then discard
previous frames until one with a stamp strictly earlier than the current one is
found; pair those.  Differences, all behavioural fixes:

* the worker blocks on a condition variable instead of busy-spinning;
* ``torch.load`` uses ``map_location`` (CPU-saved or GPU-saved weights work on
  either), no DataParallel wrapper is needed to strip ``module.``;
* the model runs through the HIP kernels on MI355X (``/RAFT/device: cuda``).

The ROS-independent part (``FramePairer`` and ``FlowInference``) is importable
without rospy; ``RaftRosNode`` needs rospy, sensor_msgs and cv_bridge.
"""
from __future__ import annotations

import collections
import threading
from argparse import Namespace
from typing import Any, Callable, Optional, Tuple

import numpy as np
import torch

from ..models import RAFT
from ..runtime import GraphedRAFT
from ..utils import checkpoint, flow_viz
from ..utils.utils import InputPadder


def _stamp_sec(msg) -> float:
    st = msg.header.stamp
    return st.to_sec() if hasattr(st, "to_sec") else float(st)


class FramePairer:
    """Thread-safe prev/curr frame queues with the reference's pairing rule."""

    def __init__(self):
        self._prev = collections.deque()
        self._curr = collections.deque()
        self._cv = threading.Condition()
        self._closed = False

    def push_prev(self, msg) -> None:
        with self._cv:
            self._prev.append(msg)
            self._cv.notify()

    def push_curr(self, msg) -> None:
        with self._cv:
            self._curr.append(msg)
            self._cv.notify()

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()

    def try_pair(self) -> Optional[Tuple[Any, Any]]:
        """Pop one (prev, curr) pair if available (caller holds no lock)."""
        with self._cv:
            return self._pair_locked()

    def _pair_locked(self):
        if not self._curr or not self._prev:
            return None
        curr = self._curr.popleft()
        while self._prev:
            prev = self._prev.popleft()
            if _stamp_sec(prev) < _stamp_sec(curr):
                return prev, curr
        return None  # no earlier prev frame: the current frame is dropped (as in the reference)

    def wait_pair(self, timeout: Optional[float] = None):
        with self._cv:
            while not self._closed:
                pair = self._pair_locked()
                if pair is not None:
                    return pair
                if not self._cv.wait(timeout):
                    return None
            return None


class FlowInference:
    """RAFT inference on numpy HxWx3 uint8 frames -> BGR uint8 flow visualisation."""

    def __init__(self, weight_path: Optional[str], small: bool = False, device: str = "cuda", iters: int = 20,
                 mixed_precision: bool = False, hip_graph: bool = True):
        if device.startswith("cuda") and not torch.cuda.is_available():
            device = "cpu"
        self.device = torch.device(device)
        self.iters = iters
        self.args = Namespace(small=small, mixed_precision=mixed_precision, alternate_corr=False)
        self.model = RAFT(self.args)
        if weight_path:
            checkpoint.load_weights(self.model, weight_path, map_location="cpu")
        self.model.to(self.device).eval()
        # camera streams have a fixed frame size: capture the forward once, replay per pair
        self.runner = GraphedRAFT(self.model, iters=iters, enabled=hip_graph)

    @torch.inference_mode()
    def flow(self, prev: np.ndarray, curr: np.ndarray) -> torch.Tensor:
        image1 = torch.from_numpy(np.ascontiguousarray(prev, dtype=np.uint8)).permute(2, 0, 1).float()[None]
        image2 = torch.from_numpy(np.ascontiguousarray(curr, dtype=np.uint8)).permute(2, 0, 1).float()[None]
        image1, image2 = image1.to(self.device), image2.to(self.device)
        padder = InputPadder(image1.shape)
        image1, image2 = padder.pad(image1, image2)
        _, flow_up = self.runner(image1, image2)
        return flow_up

    def visualize(self, prev: np.ndarray, curr: np.ndarray) -> np.ndarray:
        """The published image: colour-coded flow of the *padded* pair, BGR uint8
        (reference convert2Img + inferRAFT, ros/scripts/main.py:70-80,117-149)."""
        flo = self.flow(prev, curr)[0].permute(1, 2, 0).float().cpu().numpy()
        rgb = flow_viz.flow_to_image(flo)
        return np.ascontiguousarray(rgb[:, :, [2, 1, 0]]).astype(np.uint8)


class RaftRosNode:
    """The ROS node; all ROS modules are injected at construction for testability."""

    def __init__(self, rospy=None, image_msg=None, cv_bridge_cls=None, inference: Optional[FlowInference] = None):
        if rospy is None:
            import rospy  # noqa: F811
        if image_msg is None:
            from sensor_msgs.msg import Image as image_msg  # noqa: F811
        if cv_bridge_cls is None:
            from cv_bridge import CvBridge as cv_bridge_cls  # noqa: F811
        self.rospy = rospy
        self.bridge = cv_bridge_cls()
        rospy.init_node("raft_ros", anonymous=True)
        self.pairer = FramePairer()
        rospy.Subscriber(rospy.get_param("/ROS/prev_img"), image_msg, self.callbackPrevImage)
        rospy.Subscriber(rospy.get_param("/ROS/curr_img"), image_msg, self.callbackCurrImage)
        self._pub = rospy.Publisher("/raft_result", image_msg, queue_size=100)
        if inference is None:
            print("Initialize RAFT...")
            inference = FlowInference(rospy.get_param("/RAFT/weight_path"), bool(rospy.get_param("/RAFT/is_small")),
                                      str(rospy.get_param("/RAFT/device")),
                                      mixed_precision=bool(_get_param(rospy, "/RAFT/mixed_precision", False)),
                                      hip_graph=bool(_get_param(rospy, "/RAFT/hip_graph", True)))
            print("Initialize RAFT finish!")
        self.inference = inference
        self._thread: Optional[threading.Thread] = None

    # reference callback names
    def callbackPrevImage(self, msg) -> None:
        self.pairer.push_prev(msg)

    def callbackCurrImage(self, msg) -> None:
        self.pairer.push_curr(msg)

    def process_pair(self, prev_msg, curr_msg):
        prev = self.bridge.imgmsg_to_cv2(prev_msg, desired_encoding="passthrough")
        curr = self.bridge.imgmsg_to_cv2(curr_msg, desired_encoding="passthrough")
        result = self.inference.visualize(np.asarray(prev), np.asarray(curr))
        header = curr_msg.header
        header.frame_id = "raft_image"
        out = self.bridge.cv2_to_imgmsg(result, encoding="passthrough", header=header)
        self._pub.publish(out)
        return out

    def thdInference(self, stop: Optional[Callable[[], bool]] = None) -> None:
        while not (stop and stop()) and not self.rospy.is_shutdown():
            pair = self.pairer.wait_pair(timeout=0.1)
            if pair is not None:
                self.process_pair(*pair)

    def start(self) -> threading.Thread:
        self._thread = threading.Thread(target=self.thdInference, daemon=True)
        self._thread.start()
        return self._thread

    def shutdown(self) -> None:
        self.pairer.close()


def _get_param(rospy, name, default):
    try:
        return rospy.get_param(name, default)
    except TypeError:  # minimal fakes without a default argument
        try:
            return rospy.get_param(name)
        except Exception:
            return default


def main():  # pragma: no cover - needs a ROS master
    import rospy

    node = RaftRosNode(rospy)
    node.start()
    rospy.spin()
    node.shutdown()
