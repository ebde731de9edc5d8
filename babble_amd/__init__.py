"""babble_amd -- MI355X-native engine for Babble's hashgraph virtual-voting path.

The compute lives in libbabble_hip.so (HIP kernels for gfx950, C ABI in
include/babble_hip.h).  `Hashgraph` mirrors the reference's Go API over that
ABI; `dag.Dag` generates the synthetic gossip DAGs the bench uses.
"""
from .hashgraph import Hashgraph, HashgraphError, comm_unique_id, shard_range  # noqa: F401

__all__ = ["Hashgraph", "HashgraphError", "comm_unique_id", "shard_range"]
