from .peer_memory import PeerAllReduce, PeerHaloExchanger1d, PeerMemoryPool

__all__ = ["PeerMemoryPool", "PeerHaloExchanger1d", "PeerAllReduce"]
