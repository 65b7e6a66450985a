"""swimhip — MI355X-native SWIM membership engine (host-side mirror of the scalecube-cluster interface).

The product is libswimhip.so (gfx950 HIP, built from ../csrc). engine() loads it and fails loudly when it is
missing or no GPU is visible. There is no CPU fallback in the product path: the CPU oracle under /oracle is test
infrastructure, and only tests and the bench's cpu_baseline leg load it.
"""
import os
from pathlib import Path

from . import _abi
from .cluster import MembershipEvent, MembershipRecord, SimulatedCluster, SwimError
from .config import ClusterConfig, SimConfig

PKG_ROOT = Path(__file__).resolve().parent.parent  # scalecube-cluster_amd/
LIB_PATH = PKG_ROOT / "csrc" / "libswimhip.so"

_lib = None


def engine():
    """Load the gfx950 engine (libswimhip.so). Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"libswimhip.so not built at {LIB_PATH}; run __graft_entry__.build()")
        _lib = _abi.load(LIB_PATH)
        if _lib.swim_abi_version() != 1:
            raise ImportError("libswimhip ABI version mismatch")
    return _lib


def cluster(cfg: SimConfig) -> SimulatedCluster:
    return SimulatedCluster(engine(), cfg)


__all__ = ["ClusterConfig", "SimConfig", "SimulatedCluster", "MembershipEvent", "MembershipRecord", "SwimError",
           "engine", "cluster", "LIB_PATH"]
