from .bottleneck import Bottleneck, FrozenBatchNorm2d, SpatialBottleneck
from .halo_exchangers import (HaloExchangerAllGather, HaloExchangerNoComm, HaloExchangerPeer, HaloExchangerSendRecv,
                              HaloPadder)

__all__ = ["Bottleneck", "SpatialBottleneck", "FrozenBatchNorm2d", "HaloExchangerNoComm", "HaloExchangerAllGather",
           "HaloExchangerSendRecv", "HaloExchangerPeer", "HaloPadder"]
