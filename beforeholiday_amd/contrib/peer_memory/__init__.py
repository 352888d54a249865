from .peer_memory import PeerHaloExchanger1d, PeerMemoryPool

__all__ = ["PeerMemoryPool", "PeerHaloExchanger1d"]
