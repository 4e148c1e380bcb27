"""gossip_amd — MI355X-native synchronous-round gossip / push-sum engine.

Host-side mirror of /root/reference/program.fs over the C ABI of libgossip_hip.so.
"""
from ._abi import ABI_VERSION, GossipError, load  # noqa: F401
from .simulator import Simulator, sizes  # noqa: F401

__all__ = ["Simulator", "sizes", "load", "GossipError", "ABI_VERSION"]
