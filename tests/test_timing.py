"""Launch timing (include/ugo_fec.h ugo_fec_timing_begin/end): the bench's
per-kernel durations come from hipExtLaunchKernel start/stop events the
library attaches to its own launches."""
import ctypes

import numpy as np
import pytest
import torch

from ugo_amd import fec


def test_timing_rejects_bad_arguments():
    lib = fec.load_library()
    assert lib.ugo_fec_timing_begin(None, 4) == 6
    assert lib.ugo_fec_timing_end(None, None, 0, None, None) == 6


@pytest.mark.gpu
def test_timing_records_each_launch_in_order(gpu):
    d, p, n, S, pitch, G = 10, 3, 13, 1350, 1360, 512
    enc = fec.New(d, p)
    sh = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device=gpu)
    masks = torch.full((G,), (1 << n) - 1 - 0b101, dtype=torch.int64, device=gpu)
    ref = sh.clone()
    enc.encode_batch(sh, S, shard_major=True)
    want = sh.clone()
    enc.timing_begin(3)
    for _ in range(2):
        enc.encode_batch(sh, S, shard_major=True)
        enc.reconstruct_batch(sh, masks, S, shard_major=True)
    recs, untimed = enc.timing_end()
    assert list(recs["kernel"]) == [1, 2, 1] and untimed == 1
    assert (recs["ms"] > 0).all() and (recs["ms"] < 50).all()
    # timed launches compute the same bytes as untimed ones
    assert torch.equal(sh[:, :, :S], want[:, :, :S])
    assert not torch.equal(want[d:, :, :S], ref[d:, :, :S])
    # timing is off again: nothing recorded without a begin
    enc.encode_batch(sh, S, shard_major=True)
    recs, untimed = enc.timing_end()
    assert len(recs) == 0 and untimed == 0


@pytest.mark.gpu
def test_timing_covers_jumbo_prepare_and_apply(gpu):
    d, p, n, S, pitch, G = 32, 8, 40, 9000, 9008, 64
    enc = fec.New(d, p)
    sh = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device=gpu)
    masks = torch.full((G,), (1 << n) - 1 - 0b11, dtype=torch.int64, device=gpu)
    enc.timing_begin(8)
    enc.encode_batch(sh, S, shard_major=True)
    enc.reconstruct_batch(sh, masks, S, shard_major=True)
    recs, untimed = enc.timing_end()
    assert list(recs["kernel"]) == [1, 3, 2] and untimed == 0


@pytest.mark.gpu
def test_wide_data_codes_run_the_vector_kernels(gpu):
    """d > 32 with at most 8 parity rows and rows of >= 64 chunks: encode and
    reconstruct run the streaming vector kernels (ids 1 and 2, after k_prepare),
    not the byte kernel (id 4)."""
    d, p, n, S, G = 40, 8, 48, 2000, 64
    enc = fec.New(d, p)
    sh = torch.randint(0, 256, (G, n, S), dtype=torch.uint8, device=gpu)
    masks = torch.full((G,), (1 << n) - 1 - 0b1011, dtype=torch.int64, device=gpu)
    enc.timing_begin(8)
    enc.encode_batch(sh, S)
    enc.reconstruct_batch(sh, masks, S)
    recs, untimed = enc.timing_end()
    assert list(recs["kernel"]) == [1, 3, 2] and untimed == 0


@pytest.mark.gpu
def test_wide_parity_codes_past_32_data_rows_stay_vectorised(gpu):
    """d > 32 with more than 8 parity rows (and short rows): the wave-aligned
    kernel folds the outputs in passes; no byte-kernel launch (id 4)."""
    d, p, n, S, G = 48, 16, 64, 256, 32
    enc = fec.New(d, p)
    sh = torch.randint(0, 256, (G, n, S), dtype=torch.uint8, device=gpu)
    masks = torch.full((G,), -1 ^ 0b111 ^ (1 << 60), dtype=torch.int64, device=gpu)
    enc.timing_begin(8)
    enc.encode_batch(sh, S)
    enc.reconstruct_batch(sh, masks, S)
    recs, untimed = enc.timing_end()
    assert list(recs["kernel"]) == [1, 3, 2] and untimed == 0
