"""ugo_amd: MI355X-native Reed-Solomon FEC for jflyup/ugo's ugo/fec.go hot path.

The package holds only what that path needs:
  csrc/        gfx950 HIP kernels + the C-ABI (built into libugofec.so)
  fec.py       host mirror of the reedsolomon.Encoder subset ugo uses
  shard.py     multi-GPU partitioning of independent packet groups
"""
from .fec import (  # noqa: F401
    Encoder,
    ErrInvShardNum,
    ErrMaxShardNum,
    ErrShardNoData,
    ErrShardSize,
    ErrTooFewShards,
    FecError,
    New,
    check_shards,
    load_library,
)

__all__ = ["Encoder", "New", "check_shards", "load_library", "FecError", "ErrInvShardNum", "ErrMaxShardNum",
           "ErrTooFewShards", "ErrShardNoData", "ErrShardSize"]
