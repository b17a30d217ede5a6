"""CPU: the C-ABI library loads, exports every symbol include/ugo_fec.h declares,
and its host-only entry points behave like the upstream checks they mirror.
No kernel is launched here."""
import ctypes

import pytest

from ugo_amd import fec


def test_library_exports_every_header_symbol():
    lib = fec.load_library()
    syms = fec.header_symbols()
    assert len(syms) >= 13, syms
    for s in syms:
        assert hasattr(lib, s), f"libugofec.so does not export {s}"


def test_abi_version_and_strerror():
    lib = fec.load_library()
    assert lib.ugo_fec_abi_version() == 9
    assert fec.strerror(3) == "too few shards given"
    assert fec.strerror(5) == "shard sizes do not match"
    assert fec.strerror(4) == "no shard data"


def test_check_shards_mirrors_upstream():
    # nil allowed (Reconstruct): empties skipped, sizes must match
    assert fec.check_shards([1350, 0, 1350], nil_ok=True) == 1350
    with pytest.raises(fec.ErrShardSize):
        fec.check_shards([1350, 0, 1350], nil_ok=False)  # Encode: empty shard is a size mismatch
    with pytest.raises(fec.ErrShardSize):
        fec.check_shards([1350, 1349], nil_ok=True)
    with pytest.raises(fec.ErrShardNoData):
        fec.check_shards([0, 0, 0], nil_ok=True)


def test_create_validates_geometry_before_touching_a_device():
    lib = fec.load_library()
    h = ctypes.c_void_p()
    assert lib.ugo_fec_create(0, 0, 3, ctypes.byref(h)) == 1   # ErrInvShardNum
    assert lib.ugo_fec_create(0, 10, -1, ctypes.byref(h)) == 1
    assert lib.ugo_fec_create(0, 200, 57, ctypes.byref(h)) == 2  # ErrMaxShardNum
    with pytest.raises(fec.ErrInvShardNum):
        fec.New(-1, 3)


def test_null_arguments_rejected():
    lib = fec.load_library()
    assert lib.ugo_fec_encode(None, None, 1, 16, 16, None) == 6
    assert lib.ugo_fec_reconstruct(None, None, None, 1, 16, 16, 0, None, None) == 6
    assert lib.ugo_fec_check_shards(0, None, 1, None) == 6
    # reconstruct_into: no context, then an empty batch (a no-op whatever the pointers)
    assert lib.ugo_fec_reconstruct_into(None, None, None, 1, 16, 16, 208, None, 16, 48, 0, None, None) == 6
    assert lib.ugo_fec_reconstruct_into(None, None, None, 0, 16, 16, 208, None, 16, 48, 0, None, None) == 6
    # the host TX route and the host paths' copy queue: no context
    assert lib.ugo_fec_set_tx_host_route(None, 0) == 6
    assert lib.ugo_fec_set_host_copy_queue(None, 1) == 6


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: a missing libugofec.so is an ImportError, not a silent
    switch to another path."""
    saved = fec._lib
    fec._lib = None
    try:
        with pytest.raises(ImportError, match="not built"):
            fec.load_library(str(tmp_path / "libugofec.so"))
    finally:
        fec._lib = saved
