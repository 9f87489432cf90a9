from .raft import RAFT  # noqa: F401
from .extractor import BasicEncoder, SmallEncoder, ResidualBlock, BottleneckBlock  # noqa: F401
from .update import (BasicUpdateBlock, SmallUpdateBlock, BasicMotionEncoder, SmallMotionEncoder,  # noqa: F401
                     ConvGRU, SepConvGRU, FlowHead)
