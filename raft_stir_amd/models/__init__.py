from .raft import RAFT
from .extractor import BasicEncoder, SmallEncoder, ResidualBlock, BottleneckBlock
from .update import (BasicUpdateBlock, SmallUpdateBlock, ConvGRU, SepConvGRU, FlowHead,
                     BasicMotionEncoder, SmallMotionEncoder)
from .corr import CorrBlock, AlternateCorrBlock

__all__ = ["RAFT", "BasicEncoder", "SmallEncoder", "ResidualBlock", "BottleneckBlock",
           "BasicUpdateBlock", "SmallUpdateBlock", "ConvGRU", "SepConvGRU", "FlowHead",
           "BasicMotionEncoder", "SmallMotionEncoder", "CorrBlock", "AlternateCorrBlock"]
