from .peer_memory import (PeerAllReduce, PeerHaloExchanger1d, PeerMemoryPool, PeerSetupError, PeerTimeoutError,
                          build_peer_allreduce)

__all__ = ["PeerMemoryPool", "PeerHaloExchanger1d", "PeerAllReduce", "PeerSetupError", "PeerTimeoutError",
           "build_peer_allreduce"]
