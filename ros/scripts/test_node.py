#!/usr/bin/env python3
"""Turns one camera topic into consecutive (prev, curr) pairs on /test_prev and /test_curr,
for exercising the inference node with a rosbag (reference ros/scripts/test_node.py)."""
import rospy
from sensor_msgs.msg import Image


class PairRepublisher:
    def __init__(self, source="/kitti/camera_color_left/image_raw"):
        rospy.init_node("test_img_pair_pub", anonymous=True)
        self.prev_pub = rospy.Publisher("/test_prev", Image, queue_size=100)
        self.curr_pub = rospy.Publisher("/test_curr", Image, queue_size=100)
        self.last = None
        rospy.Subscriber(rospy.get_param("~source", source), Image, self.on_image)

    def on_image(self, msg):
        if self.last is not None:
            self.prev_pub.publish(self.last)
            self.curr_pub.publish(msg)
        self.last = msg


if __name__ == "__main__":
    PairRepublisher()
    rospy.spin()
