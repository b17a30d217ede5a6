"""Multi-GPU partitioning of packet groups.

Every ugo FEC packet group (ugo/fec.go:145-146: group = seqid / (d+p)) is an
independent codeword, so a batch shards across GPUs by contiguous group ranges
with no data-path collective.  One process per GPU; the only cross-rank
traffic is the timing barrier and the max-over-ranks reduction in bench.py.
"""
from __future__ import annotations

from typing import Tuple


def partition(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced range [g0, g1) of `total` groups for `rank`."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} / world {world}")
    return total * rank // world, total * (rank + 1) // world


def dist_env():
    """(rank, local_rank, world_size) from the torchrun environment."""
    import os

    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))
