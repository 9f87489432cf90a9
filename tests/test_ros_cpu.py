"""ROS node with fake rospy / sensor_msgs / cv_bridge (ROS is not installed here)."""
import threading
import types

import numpy as np
import pytest

from raft_ros_amd.ros.node import FlowInference, FramePairer, RaftRosNode


class Stamp:
    def __init__(self, t):
        self.t = t

    def to_sec(self):
        return self.t


class Header:
    def __init__(self, t):
        self.stamp = Stamp(t)
        self.frame_id = "camera"


class Msg:
    def __init__(self, t, img=None):
        self.header = Header(t)
        self.img = img


class FakeRospy(types.SimpleNamespace):
    def __init__(self, params):
        super().__init__(params=params, subs={}, pubs=[], inited=None)

    def init_node(self, name, anonymous=False):
        self.inited = name

    def get_param(self, name, default=None):
        return self.params.get(name, default)

    def Subscriber(self, topic, typ, cb):
        self.subs[topic] = cb

    def Publisher(self, topic, typ, queue_size=None):
        pub = types.SimpleNamespace(topic=topic, queue_size=queue_size, sent=[])
        pub.publish = pub.sent.append
        self.pubs.append(pub)
        return pub

    def is_shutdown(self):
        return False


class FakeBridge:
    def imgmsg_to_cv2(self, msg, desired_encoding="passthrough"):
        return msg.img

    def cv2_to_imgmsg(self, img, encoding="passthrough", header=None):
        return types.SimpleNamespace(data=img, encoding=encoding, header=header)


def test_pairing_rule():
    p = FramePairer()
    for t in (1.0, 2.0, 3.0):
        p.push_prev(Msg(t))
    p.push_curr(Msg(2.5))
    prev, curr = p.try_pair()
    assert prev.header.stamp.t == 1.0 and curr.header.stamp.t == 2.5  # oldest earlier prev
    p.push_curr(Msg(1.5))  # remaining prevs (2.0, 3.0) are not earlier: consumed and dropped
    assert p.try_pair() is None
    assert p.try_pair() is None


def test_wait_pair_blocks_until_data():
    p = FramePairer()
    out = []
    th = threading.Thread(target=lambda: out.append(p.wait_pair(timeout=5)))
    th.start()
    p.push_curr(Msg(2.0))
    p.push_prev(Msg(1.0))
    th.join(5)
    assert out and out[0][0].header.stamp.t == 1.0


@pytest.fixture(scope="module")
def small_inference():
    return FlowInference(None, small=True, device="cpu", iters=2)


def test_node_publishes_padded_bgr_flow(small_inference):
    rospy = FakeRospy({"/ROS/prev_img": "/test_prev", "/ROS/curr_img": "/test_curr"})
    node = RaftRosNode(rospy, image_msg=object, cv_bridge_cls=FakeBridge, inference=small_inference)
    assert rospy.inited == "raft_ros" and set(rospy.subs) == {"/test_prev", "/test_curr"}
    pub = rospy.pubs[0]
    assert pub.topic == "/raft_result" and pub.queue_size == 100
    img = (np.random.rand(130, 150, 3) * 255).astype(np.uint8)
    rospy.subs["/test_prev"](Msg(1.0, img))
    rospy.subs["/test_curr"](Msg(2.0, img))
    stop = {"n": 0}

    def done():
        stop["n"] += 1
        return bool(pub.sent) or stop["n"] > 50

    node.thdInference(stop=done)
    assert len(pub.sent) == 1
    out = pub.sent[0]
    assert out.encoding == "passthrough" and out.header.frame_id == "raft_image" and out.header.stamp.t == 2.0
    assert out.data.shape == (136, 152, 3) and out.data.dtype == np.uint8  # padded to /8, like the reference


def test_flow_inference_matches_model_on_static_pair(small_inference):
    img = (np.random.rand(128, 128, 3) * 255).astype(np.uint8)
    vis = small_inference.visualize(img, img)
    assert vis.shape == (128, 128, 3)
