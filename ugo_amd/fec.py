"""Python host mirror of the reedsolomon.Encoder subset used by jflyup/ugo.

ugo/fec.go drives klauspost/reedsolomon through three calls:
  reedsolomon.New(dataShards, parityShards)   ugo/fec.go:59
  enc.Reconstruct(shards)                     ugo/fec.go:202
  enc.Encode(shards)                          ugo/fec.go:238
This module exposes the same names and argument meaning over the C-ABI in
include/ugo_fec.h (libugofec.so, gfx950 kernels):

* ``New(d, p, device=0)`` -> ``Encoder`` (raises ``ErrInvShardNum`` /
  ``ErrMaxShardNum`` like upstream ``New``).
* ``Encoder.Encode(shards)`` / ``Encoder.Reconstruct(shards)`` /
  ``Encoder.ReconstructData(shards)``: Go-shaped, one group per call, shards
  are a list of ``bytearray`` (``None`` or empty = missing), same error
  behaviour (``ErrTooFewShards``, ``ErrShardNoData``, ``ErrShardSize``).
* ``Encoder.encode_batch`` / ``reconstruct_batch``: the device-resident batch
  form (torch uint8 tensors on the GPU, shape [groups, d+p, pitch]).
* ``Encoder.encode_host`` / ``reconstruct_host``: host numpy batches, staged
  through the engine's pipelined H2D -> kernel -> D2H path.

There is no CPU fallback: if libugofec.so is missing the import fails, and
every compute call needs a gfx950 device.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import List, Optional, Sequence

import numpy as np

try:  # load torch first so libugofec.so binds torch's libamdhip64.so.7 (same soname)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host-only paths
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# UGO_FEC_LIB: another build of the same library (interleaved A/B runs in tools/)
LIB_PATH = os.environ.get("UGO_FEC_LIB") or os.path.join(_HERE, "libugofec.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ugo_fec.h")
CONN_HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ugo_fec_conn.h")
PKT_HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ugo_pkt.h")

OK = 0
RECONSTRUCT_DATA_ONLY = 1


class FecError(Exception):
    code = -1


class ErrInvShardNum(FecError):
    code = 1


class ErrMaxShardNum(FecError):
    code = 2


class ErrTooFewShards(FecError):
    code = 3


class ErrShardNoData(FecError):
    code = 4


class ErrShardSize(FecError):
    code = 5


class ErrInvalidArg(FecError):
    code = 6


class ErrSingular(FecError):
    code = 7


class ErrHip(FecError):
    code = 8


class ErrNoDevice(FecError):
    code = 9


_ERRORS = {c.code: c for c in (ErrInvShardNum, ErrMaxShardNum, ErrTooFewShards, ErrShardNoData,
                                ErrShardSize, ErrInvalidArg, ErrSingular, ErrHip, ErrNoDevice)}

_lib = None

# include/ugo_pkt.h
PKT_FEC_FRAMED = 1
PKT_INFO_DTYPE = np.dtype([("packet_number", "<u8"), ("stop_waiting", "<u8"), ("largest_acked", "<u8"),
                           ("largest_in_order", "<u8"), ("delay_us", "<u8"), ("status", "<u4"),
                           ("payload_off", "<u4"), ("n_ranges", "<u2"), ("n_segments", "<u2"), ("flags", "u1"),
                           ("fec_flag_lo", "u1"), ("reserved", "u1", (10,))])
# include/ugo_fec.h launch timing
KERNEL_NAMES = {1: "encode", 2: "reconstruct", 3: "prepare", 4: "bytes", 5: "rx_assemble", 6: "tx_assemble",
                7: "packet_decode"}
KERNEL_IDS = {v: k for k, v in KERNEL_NAMES.items()}
LAUNCH_TIME_DTYPE = np.dtype([("kernel", "<u4"), ("ms", "<f4")])
PKT_SEGMENT_DTYPE = np.dtype([("offset", "<u8"), ("data_off", "<u4"), ("len", "<u2"), ("avail", "<u2")])
assert PKT_INFO_DTYPE.itemsize == 64 and PKT_SEGMENT_DTYPE.itemsize == 16


def load_library(path: str = LIB_PATH):
    """Load libugofec.so.  Raises loudly if it was not built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run `make -C ugo_amd/csrc` (or __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    sz, vp, i, u = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint
    lib.ugo_fec_create.argtypes = [i, i, i, ctypes.POINTER(vp)]
    lib.ugo_fec_destroy.argtypes = [vp]
    lib.ugo_fec_destroy.restype = None
    lib.ugo_fec_geometry.argtypes = [vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)]
    lib.ugo_fec_matrix.argtypes = [vp, vp]
    lib.ugo_fec_encode.argtypes = [vp, vp, sz, sz, sz, vp]
    lib.ugo_fec_reconstruct.argtypes = [vp, vp, vp, sz, sz, sz, u, vp, vp]
    lib.ugo_fec_encode_strided.argtypes = [vp, vp, sz, sz, sz, sz, vp]
    lib.ugo_fec_reconstruct_strided.argtypes = [vp, vp, vp, sz, sz, sz, sz, u, vp, vp]
    lib.ugo_fec_reconstruct_into.argtypes = [vp, vp, vp, sz, sz, sz, sz, vp, sz, sz, u, vp, vp]
    lib.ugo_fec_encode_host.argtypes = [vp, vp, sz, sz, sz]
    lib.ugo_fec_reconstruct_host.argtypes = [vp, vp, vp, sz, sz, sz, u, vp]
    lib.ugo_fec_service_start.argtypes = [vp, u]
    lib.ugo_fec_service_stop.argtypes = [vp]
    lib.ugo_fec_service_config.argtypes = [vp, u, u, u]
    lib.ugo_fec_poisoned.argtypes = [vp]
    lib.ugo_fec_check_shards.argtypes = [i, vp, i, ctypes.POINTER(sz)]
    lib.ugo_fec_host_alloc.argtypes = [sz, ctypes.POINTER(vp)]
    lib.ugo_fec_host_free.argtypes = [vp]
    lib.ugo_fec_strerror.argtypes = [i]
    lib.ugo_fec_strerror.restype = ctypes.c_char_p
    lib.ugo_fec_abi_version.argtypes = []
    lib.ugo_fec_rx_assemble.argtypes = [vp, vp, sz, vp, sz, vp, ctypes.c_uint64, sz, vp, sz, sz, sz, vp, vp, vp]
    lib.ugo_fec_rx_assemble_frames.argtypes = lib.ugo_fec_rx_assemble.argtypes
    lib.ugo_fec_rc4_keystream.argtypes = [vp, sz, vp, sz]
    lib.ugo_fec_tx_assemble.argtypes = [vp, vp, sz, vp, sz, ctypes.c_uint32, vp, sz, vp, sz, vp, vp, vp]
    lib.ugo_fec_packet_decode.argtypes = [vp, vp, sz, vp, sz, vp, u, vp, vp, sz, vp, sz, vp]
    lib.ugo_fec_reconstruct_rows.argtypes = [vp, vp, vp, sz, sz, vp, sz, sz, u, vp, vp]
    lib.ugo_fec_lossy_groups.argtypes = [vp, vp, sz, u, vp, vp, vp]
    lib.ugo_fec_rx_recover_host.argtypes = [vp, vp, sz, vp, sz, vp, ctypes.c_uint64, sz, sz, vp, vp, vp, sz, sz, vp,
                                            ctypes.POINTER(sz)]
    lib.ugo_fec_tx_assemble_host.argtypes = [vp, vp, sz, vp, sz, ctypes.c_uint32, vp, sz, vp, sz, vp, vp]
    lib.ugo_fec_set_tx_host_route.argtypes = [vp, ctypes.c_int]
    lib.ugo_fec_set_host_copy_queue.argtypes = [vp, ctypes.c_int]
    lib.ugo_fec_reconstruct_list.argtypes = [vp, vp, vp, sz, vp, vp, sz, sz, sz, sz, vp, sz, sz, u, vp, vp]
    lib.ugo_fec_recover_data.argtypes = [vp, vp, vp, sz, sz, sz, sz, vp, sz, sz, vp, vp, vp]
    lib.ugo_fec_device_address.argtypes = [vp, vp, ctypes.POINTER(vp)]
    lib.ugo_fec_timing_begin.argtypes = [vp, sz]
    lib.ugo_fec_timing_end.argtypes = [vp, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    _lib = lib
    return lib


def header_symbols(paths=(HEADER_PATH, CONN_HEADER_PATH, PKT_HEADER_PATH)) -> List[str]:
    """Every entry point declared in include/ugo_fec.h, ugo_fec_conn.h and ugo_pkt.h."""
    out = set()
    for path in paths:
        src = open(path).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        out |= set(re.findall(r"\b(ugo_fec(?:conn)?_[a-z0-9_]+)\s*\(", src))
    return sorted(out)


def strerror(code: int) -> str:
    return load_library().ugo_fec_strerror(code).decode()


def _require(cond, msg: str = "argument does not match the batch layout the entry point expects"):
    """Argument checks that guard device memory (sizes the kernels index by):
    explicit, so they hold under `python -O` too."""
    if not cond:
        raise ValueError(msg)


def _raise(code: int):
    if code != OK:
        raise _ERRORS.get(code, FecError)(f"{strerror(code)} (status {code})")


def check_shards(lens: Sequence[int], nil_ok: bool) -> int:
    """klauspost checkShards over shard lengths; returns the shard size."""
    lib = load_library()
    arr = (ctypes.c_size_t * len(lens))(*lens)
    out = ctypes.c_size_t(0)
    _raise(lib.ugo_fec_check_shards(len(lens), ctypes.cast(arr, ctypes.c_void_p), int(nil_ok),
                                    ctypes.byref(out)))
    return out.value


def _stream_handle(stream) -> Optional[int]:
    if stream is None and torch is not None and torch.cuda.is_available():
        stream = torch.cuda.current_stream()
    if stream is None:
        return None
    return int(getattr(stream, "cuda_stream", stream))


class Encoder:
    """A (d, p) code bound to one GPU (reedsolomon.Encoder equivalent)."""

    def __init__(self, data_shards: int, parity_shards: int, device: int = 0):
        lib = load_library()
        h = ctypes.c_void_p()
        _raise(lib.ugo_fec_create(device, data_shards, parity_shards, ctypes.byref(h)))
        self._h = h
        self.DataShards = data_shards
        self.ParityShards = parity_shards
        self.Shards = data_shards + parity_shards
        self.mask_words = (self.Shards + 63) // 64  # presence words per group (include/ugo_fec.h)
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            load_library().ugo_fec_destroy(self._h)
            self._h = None
        if getattr(self, "_stage_buf", None) is not None:
            host_free(self._stage_buf)
            self._stage_buf = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def matrix(self) -> np.ndarray:
        out = np.zeros((self.Shards, self.DataShards), np.uint8)
        _raise(load_library().ugo_fec_matrix(self._h, out.ctypes.data))
        return out

    # -------------------------------------------------- device-resident batch
    def _geom(self, shards, shard_major: bool):
        """(groups, pitch, row_stride, group_stride) of a uint8 tensor whose
        last dimension is contiguous: group-major [G, d+p, pitch] or
        shard-major [d+p, G, pitch] (planar); the row and group strides are the
        tensor's own (a padded row stride is a strided view)."""
        _require(shards.dim() == 3 and shards.element_size() == 1 and shards.stride(2) == 1)
        if shard_major:
            n, G, pitch = shards.shape
            rs, gs = shards.stride(0), shards.stride(1)
        else:
            G, n, pitch = shards.shape
            gs, rs = shards.stride(0), shards.stride(1)
        _require(n == self.Shards, f"expected {self.Shards} rows per group, got {n}")
        return G, pitch, rs, gs

    def encode_batch(self, shards, shard_size: Optional[int] = None, stream=None, shard_major: bool = False):
        """Encode every group of a device tensor: [G, d+p, pitch] (default) or,
        with shard_major=True, the planar [d+p, G, pitch] layout."""
        G, pitch, rs, gs = self._geom(shards, shard_major)
        S = pitch if shard_size is None else shard_size
        _raise(load_library().ugo_fec_encode_strided(self._h, shards.data_ptr(), G, S, rs, gs,
                                                     _stream_handle(stream)))

    def reconstruct_batch(self, shards, present, shard_size: Optional[int] = None, data_only=False,
                          status=None, stream=None, shard_major: bool = False):
        """present: int64/uint64 CUDA tensor [G] of presence bitmasks (bit r = shard r
        non-empty), [G][W] words for d+p > 64 (W = mask_words); status: optional int8
        CUDA tensor [G]."""
        G, pitch, rs, gs = self._geom(shards, shard_major)
        _require(present.is_contiguous() and present.numel() == G * self.mask_words and present.element_size() == 8)
        S = pitch if shard_size is None else shard_size
        st = None if status is None else status.data_ptr()
        _raise(load_library().ugo_fec_reconstruct_strided(self._h, shards.data_ptr(), present.data_ptr(), G, S, rs,
                                                          gs, RECONSTRUCT_DATA_ONLY if data_only else 0, st,
                                                          _stream_handle(stream)))

    def reconstruct_into(self, shards, present, out, shard_size: Optional[int] = None, data_only=False,
                         status=None, stream=None, shard_major: bool = False, out_shard_major: bool = True):
        """Reconstruct with a separate output batch (include/ugo_fec.h
        ugo_fec_reconstruct_into): `shards` is only read; output i of group g (the
        i-th erased row, ascending) goes to `out`, a contiguous uint8 CUDA tensor
        [p][G][opitch] (out_shard_major) or [G][p][opitch]."""
        G, pitch, rs, gs = self._geom(shards, shard_major)
        _require(present.is_contiguous() and present.numel() == G * self.mask_words and present.element_size() == 8)
        _require(out.is_contiguous() and out.element_size() == 1 and out.dim() == 3)
        p = self.ParityShards
        if out_shard_major:
            _require(out.shape[0] == p and out.shape[1] == G)
            opitch = out.shape[2]
            ors, ogs = G * opitch, opitch
        else:
            _require(out.shape[0] == G and out.shape[1] == p)
            opitch = out.shape[2]
            ors, ogs = opitch, p * opitch
        S = pitch if shard_size is None else shard_size
        _require(opitch >= S)
        st = None if status is None else status.data_ptr()
        _raise(load_library().ugo_fec_reconstruct_into(self._h, shards.data_ptr(), present.data_ptr(), G, S, rs, gs,
                                                       out.data_ptr(), ors, ogs,
                                                       RECONSTRUCT_DATA_ONLY if data_only else 0, st,
                                                       _stream_handle(stream)))

    def lossy_groups(self, present, data_only: bool = True, out=None, count=None, stream=None):
        """ugo_fec_lossy_groups: the groups of `present` (int64 CUDA [G]) with an
        erased row to rebuild (data rows only with data_only), ascending.  Returns
        (list, count): an int32 CUDA tensor [G] whose first *count entries are the
        groups, and an int32 CUDA tensor [1]; nothing is synchronised."""
        import torch

        G = present.numel()
        _require(present.is_contiguous() and present.element_size() == 8 and self.mask_words == 1)
        lst = torch.empty(max(G, 1), dtype=torch.int32, device=present.device) if out is None else out
        cnt = torch.empty(1, dtype=torch.int32, device=present.device) if count is None else count
        _require(lst.numel() >= G and lst.element_size() == 4 and cnt.element_size() == 4)
        _raise(load_library().ugo_fec_lossy_groups(self._h, present.data_ptr(), G,
                                                   RECONSTRUCT_DATA_ONLY if data_only else 0, lst.data_ptr(),
                                                   cnt.data_ptr(), _stream_handle(stream)))
        return lst, cnt

    def reconstruct_list(self, shards, present, lst, count, out, shard_size: Optional[int] = None,
                         data_only: bool = True, status=None, stream=None, shard_major: bool = True,
                         max_entries: Optional[int] = None):
        """ugo_fec_reconstruct_list: Reconstruct the groups lst[0 .. *count) of the
        batch; output i of list entry j goes to out[j, i] (out: contiguous uint8
        CUDA tensor [max_entries][slots][opitch], compact in list order) or, out =
        None, in place.  status: int8 CUDA [max_entries] (entry j's status)."""
        G, pitch, rs, gs = self._geom(shards, shard_major)
        _require(present.is_contiguous() and present.numel() == G and present.element_size() == 8)
        m = G if max_entries is None else max_entries
        S = pitch if shard_size is None else shard_size
        ors = oes = 0
        if out is not None:
            _require(out.is_contiguous() and out.element_size() == 1 and out.dim() == 3 and out.shape[0] >= m)
            ors, oes = out.shape[2], out.shape[1] * out.shape[2]
            _require(out.shape[2] >= S)
        _raise(load_library().ugo_fec_reconstruct_list(
            self._h, shards.data_ptr(), present.data_ptr(), G, lst.data_ptr(), count.data_ptr(), m, S, rs, gs,
            None if out is None else out.data_ptr(), ors, oes, RECONSTRUCT_DATA_ONLY if data_only else 0,
            None if status is None else status.data_ptr(), _stream_handle(stream)))

    def recover_data(self, shards, present, out, index, count=None, shard_size: Optional[int] = None,
                     stream=None, shard_major: bool = True):
        """ugo_fec_recover_data: `input`'s recovered data shards of a device batch,
        row-compact in `recovered` order: out[r, :shard_size] (out: contiguous
        uint8 CUDA [max_rows, row]), index[r] = group*(d+p) + row (int32 CUDA
        [max_rows]); returns count (int32 CUDA [1], the number recovered,
        written on the stream)."""
        import torch

        G, pitch, rs, gs = self._geom(shards, shard_major)
        _require(present.is_contiguous() and present.numel() == G and present.element_size() == 8)
        S = pitch if shard_size is None else shard_size
        _require(out.is_contiguous() and out.element_size() == 1 and out.dim() == 2 and out.shape[1] >= S)
        _require(index.is_contiguous() and index.element_size() == 4 and index.numel() >= out.shape[0])
        cnt = torch.empty(1, dtype=torch.int32, device=present.device) if count is None else count
        _raise(load_library().ugo_fec_recover_data(
            self._h, shards.data_ptr(), present.data_ptr(), G, S, rs, gs, out.data_ptr(), out.shape[1], out.shape[0],
            index.data_ptr(), cnt.data_ptr(), _stream_handle(stream)))
        return cnt

    def rx_recover_host(self, wire: np.ndarray, lens: np.ndarray, shard_size: int, groups: int,
                        first_group: int = 0, pad: Optional[bytes] = None, out: Optional[np.ndarray] = None,
                        max_out: Optional[int] = None, present_out: Optional[np.ndarray] = None):
        """ugo_fec_rx_recover_host: the RX path host memory to host memory.  wire =
        uint8 [npk, slot] (pinned for DMA rates), lens = uint16 [npk].  Returns
        (n, index, out, stats): n recovered data shards, the first
        min(n, max_out) of them row-compact in out[r, :shard_size] (out: uint8
        [max_out, row] with row >= shard_size, allocated if None) in ugo's
        `recovered` order, index[r] = window group * (d+p) + row."""
        npk, slot = wire.shape
        _require(wire.flags.c_contiguous and wire.itemsize == 1)
        _require(lens.flags.c_contiguous and lens.size == npk and lens.itemsize == 2)
        _require(pad is None or len(pad) >= slot, "pad must hold at least slot_stride keystream bytes")
        if present_out is not None:  # C writes groups * 8 bytes there
            _require(isinstance(present_out, np.ndarray) and present_out.flags.c_contiguous
                     and present_out.itemsize == 8 and present_out.size >= groups)
        m = groups * min(self.DataShards, self.ParityShards) if max_out is None else max_out
        if out is None:
            out = np.zeros((max(m, 1), (shard_size + 15) // 16 * 16), np.uint8)
        _require(out.ndim == 2 and out.flags.c_contiguous and out.shape[0] >= m and out.shape[1] >= shard_size)
        index = np.zeros(max(m, 1), np.uint32)
        stats = np.zeros(5, np.uint32)
        padb = None if pad is None else np.frombuffer(bytes(pad), np.uint8)
        n_out = ctypes.c_size_t(0)
        _raise(load_library().ugo_fec_rx_recover_host(
            self._h, wire.ctypes.data, slot, lens.ctypes.data, npk, None if padb is None else padb.ctypes.data,
            first_group, groups, shard_size, None if present_out is None else present_out.ctypes.data,
            stats.ctypes.data, out.ctypes.data, out.shape[1], m, index.ctypes.data, ctypes.byref(n_out)))
        return n_out.value, index, out, stats

    def tx_assemble_host(self, pkts: np.ndarray, lens: np.ndarray, wire: np.ndarray, wire_lens: np.ndarray,
                         first_seq: int = 0, pad: Optional[bytes] = None, max_len: int = 1476,
                         status: Optional[np.ndarray] = None):
        """ugo_fec_tx_assemble_host: tx_assemble with host numpy buffers (pinned for
        DMA rates): pkts uint8 [G*d, slot_in], lens uint16 [G*d], wire uint8
        [G*(d+p), slot_out], wire_lens uint16 [G*(d+p)], status int8 [G] or None."""
        d, n = self.DataShards, self.Shards
        _require(pkts.ndim == 2 and wire.ndim == 2 and pkts.shape[0] % d == 0)
        G = pkts.shape[0] // d
        _require(lens.size == G * d and wire.shape[0] == G * n and wire_lens.size == G * n)
        # the C side copies G*d*2, G*n*2 and G bytes and reads round_up(max_len, 16) pad bytes
        for a in (pkts, wire, lens, wire_lens):
            _require(isinstance(a, np.ndarray) and a.flags.c_contiguous)
        _require(pkts.itemsize == 1 and wire.itemsize == 1 and lens.itemsize == 2 and wire_lens.itemsize == 2)
        if status is not None:
            _require(isinstance(status, np.ndarray) and status.flags.c_contiguous and status.size == G
                     and status.itemsize == 1)
        _require(pad is None or len(pad) >= (max_len + 15) // 16 * 16,
                 "pad must hold at least round_up(max_len, 16) keystream bytes")
        padb = None if pad is None else np.frombuffer(bytes(pad), np.uint8)
        _raise(load_library().ugo_fec_tx_assemble_host(
            self._h, pkts.ctypes.data, pkts.shape[1], lens.ctypes.data, G, first_seq,
            None if padb is None else padb.ctypes.data, max_len, wire.ctypes.data, wire.shape[1],
            wire_lens.ctypes.data, None if status is None else status.ctypes.data))

    def set_host_copy_queue(self, on: bool):
        """ugo_fec_set_host_copy_queue: the host paths' H2D copies on a
        low-priority stream (a hardware-queue pool of its own)."""
        _raise(load_library().ugo_fec_set_host_copy_queue(self._h, 1 if on else 0))

    def set_tx_host_route(self, route: str):
        """ugo_fec_set_tx_host_route: tx_assemble_host's wire packets by D2H
        copy ("copy", the default) or written through the pinned buffer's
        mapping ("mapped")."""
        _require(route in ("copy", "mapped"))
        _raise(load_library().ugo_fec_set_tx_host_route(self._h, {"copy": 0, "mapped": 1}[route]))

    def reconstruct_rows(self, rows, present, out, shard_size: int, data_only=False, status=None, stream=None,
                         out_shard_major: bool = True):
        """Reconstruct from a row-pointer table (include/ugo_fec.h
        ugo_fec_reconstruct_rows): rows = int64 tensor [G, d+p] of device
        addresses (device tensor, or pinned host memory as a numpy array /
        CPU tensor viewed through ugo_fec_device_address), present = [G] masks
        (device tensor or pinned numpy array), out = contiguous uint8 CUDA
        tensor [p][G][opitch] (out_shard_major) or [G][p][opitch]."""
        G = present.shape[0]
        _require(rows.shape[0] == G and rows.shape[1] == self.Shards and self.Shards <= 64)
        p = self.ParityShards
        _require(out.dim() == 3 and out.is_contiguous() and out.element_size() == 1)
        if out_shard_major:
            _require(out.shape[0] == p and out.shape[1] == G)
            ors, ogs = G * out.shape[2], out.shape[2]
        else:
            _require(out.shape[0] == G and out.shape[1] == p)
            ors, ogs = out.shape[2], p * out.shape[2]
        _require(out.shape[2] >= shard_size)

        def ptr(x):
            return None if x is None else (x.ctypes.data if isinstance(x, np.ndarray) else x.data_ptr())

        _raise(load_library().ugo_fec_reconstruct_rows(self._h, ptr(rows), ptr(present), G, shard_size, ptr(out),
                                                       ors, ogs, RECONSTRUCT_DATA_ONLY if data_only else 0,
                                                       ptr(status), _stream_handle(stream)))

    def device_address(self, addr: int) -> int:
        """ugo_fec_device_address: the device address of host/device pointer addr."""
        out = ctypes.c_void_p()
        _raise(load_library().ugo_fec_device_address(self._h, ctypes.c_void_p(addr), ctypes.byref(out)))
        return out.value or 0

    def rx_assemble(self, wire, lens, shards, present, first_group: int = 0, shard_size: Optional[int] = None,
                    pad=None, stats=None, stream=None, shard_major: bool = True, frames: bool = False):
        """RX group assembly (include/ugo_fec.h ugo_fec_rx_assemble): wire = uint8 CUDA
        tensor [npk, slot] of received packets, lens = int16/uint16 CUDA tensor [npk];
        pad = uint8 CUDA keystream (>= slot bytes) or None; present = int64 CUDA [G]
        (zeroed by the caller); stats = int32 CUDA [5] (accepted, bad flag, out of
        window, too short, duplicate) or None.  A repeated seqid keeps its first
        copy in ring order (ugo/fec.go:123-129).  frames=True:
        ugo_fec_rx_assemble_frames -- a row holds the decrypted packet (payload at
        column 6, shard_size + 6 bytes); reconstruct it with shard_size + 6."""
        if stats is not None:
            _require(stats.numel() >= 5 and stats.element_size() == 4)
        G, pitch, rs, gs = self._geom(shards, shard_major)
        npk, slot = wire.shape
        _require(wire.is_contiguous() and lens.is_contiguous() and lens.element_size() == 2 and lens.numel() == npk)
        S = (pitch - 6 if frames else pitch) if shard_size is None else shard_size
        if pad is not None:
            _require(pad.is_contiguous() and pad.element_size() == 1 and pad.numel() >= slot)
        entry = load_library().ugo_fec_rx_assemble_frames if frames else load_library().ugo_fec_rx_assemble
        _raise(entry(
            self._h, wire.data_ptr(), slot, lens.data_ptr(), npk, None if pad is None else pad.data_ptr(),
            first_group, G, shards.data_ptr(), S, rs, gs, present.data_ptr(),
            None if stats is None else stats.data_ptr(), _stream_handle(stream)))

    def tx_assemble(self, pkts, lens, wire, wire_lens, first_seq: int = 0, pad=None, max_len: int = 1476,
                    status=None, stream=None):
        """TX group assembly (include/ugo_fec.h ugo_fec_tx_assemble): pkts = uint8 CUDA
        tensor [G*d, slot_in] of outgoing data packets (6-B header space first),
        lens = int16/uint16 CUDA [G*d]; wire = uint8 CUDA [G*(d+p), slot_out],
        wire_lens = int16/uint16 CUDA [G*(d+p)]; pad = uint8 CUDA keystream or None;
        status = int8 CUDA [G] or None."""
        d, n = self.DataShards, self.Shards
        npk, slot_in = pkts.shape
        _require(npk % d == 0, "pkts must hold whole groups of d data packets")
        G = npk // d
        _require(wire.shape[0] == G * n and wire_lens.numel() == G * n and lens.numel() == npk)
        _require(pkts.is_contiguous() and wire.is_contiguous() and lens.is_contiguous() and wire_lens.is_contiguous())
        _require(lens.element_size() == 2 and wire_lens.element_size() == 2)
        if status is not None:
            _require(status.numel() == G and status.element_size() == 1)
        _raise(load_library().ugo_fec_tx_assemble(
            self._h, pkts.data_ptr(), slot_in, lens.data_ptr(), G, first_seq,
            None if pad is None else pad.data_ptr(), max_len, wire.data_ptr(), wire.shape[1],
            wire_lens.data_ptr(), None if status is None else status.data_ptr(), _stream_handle(stream)))

    def packet_decode(self, pkts, lens, pad=None, framed: bool = False, max_ranges: int = 32,
                      max_segments: int = 8, stream=None, out=None):
        """Batch ugoPacket.decode (include/ugo_pkt.h): pkts = uint8 CUDA [npk, slot],
        lens = int16/uint16 CUDA [npk].  Returns CUDA tensors (info [npk, 64] bytes --
        view on the host with PKT_INFO_DTYPE --, ranges int64 [npk, max_ranges, 2],
        segs [npk, max_segments, 16] bytes -- PKT_SEGMENT_DTYPE)."""
        npk, slot = pkts.shape
        _require(pkts.is_contiguous() and lens.is_contiguous() and lens.element_size() == 2 and lens.numel() == npk)
        dev = pkts.device
        if out is not None:  # reuse (info, ranges, segs) from an earlier call
            info, ranges, segs = out
            _require(info.shape == (npk, 64) and ranges.shape[0] == npk and segs.shape[0] == npk)
            _require(ranges.shape[1] >= max(max_ranges, 1) and segs.shape[1] >= max(max_segments, 1))
        else:
            info = torch.empty((npk, 64), dtype=torch.uint8, device=dev)
            ranges = torch.zeros((npk, max(max_ranges, 1), 2), dtype=torch.int64, device=dev)
            segs = torch.zeros((npk, max(max_segments, 1), 16), dtype=torch.uint8, device=dev)
        _raise(load_library().ugo_fec_packet_decode(
            self._h, pkts.data_ptr(), slot, lens.data_ptr(), npk, None if pad is None else pad.data_ptr(),
            PKT_FEC_FRAMED if framed else 0, info.data_ptr(), ranges.data_ptr(), max_ranges, segs.data_ptr(),
            max_segments, _stream_handle(stream)))
        return info, ranges, segs

    # ---------------------------------------------------------- launch timing
    def timing_begin(self, max_launches: int):
        """Time the next max_launches kernel launches of this context with
        hipExtLaunchKernel start/stop events (kernel durations, nothing inserted
        between kernels).  Read them with timing_end()."""
        _raise(load_library().ugo_fec_timing_begin(self._h, max_launches))
        self._timing_cap = max_launches

    def timing_end(self):
        """Waits for the timed launches; returns (records, untimed): records is a
        LAUNCH_TIME_DTYPE array (kernel id, ms) in launch order, untimed the
        number of launches past max_launches."""
        cap = getattr(self, "_timing_cap", 0)
        out = np.zeros(cap, LAUNCH_TIME_DTYPE)
        n, untimed = ctypes.c_size_t(), ctypes.c_size_t()
        _raise(load_library().ugo_fec_timing_end(self._h, out.ctypes.data if cap else None, cap, ctypes.byref(n),
                                                 ctypes.byref(untimed)))
        return out[:n.value], untimed.value

    # ------------------------------------------------------ host-buffer batch
    def service_start(self, idle_us: int = 0):
        """Per-call latency service (ugo_fec_service_start): small pinned host
        batches are served by a resident workgroup, no launch per call."""
        _raise(load_library().ugo_fec_service_start(self._h, idle_us))

    def service_stop(self):
        _raise(load_library().ugo_fec_service_stop(self._h))

    def service_config(self, timeout_ms: int = 0, grace_ms: int = 0, test_stall_us: int = 0):
        """The service's watchdog (ugo_fec_service_config): a call's wait for an
        answer and the wait for the workgroup to leave after a timeout (0 = 5000
        ms each); test_stall_us (tests only) delays every request it serves."""
        _raise(load_library().ugo_fec_service_config(self._h, timeout_ms, grace_ms, test_stall_us))

    @property
    def poisoned(self) -> bool:
        """True if a service workgroup never left after a failed call (every call
        on this context now fails; include/ugo_fec.h)."""
        return bool(load_library().ugo_fec_poisoned(self._h))

    def encode_host(self, shards: np.ndarray, shard_size: Optional[int] = None):
        _require(shards.dtype == np.uint8 and shards.flags["C_CONTIGUOUS"] and shards.ndim == 3)
        G, n, pitch = shards.shape
        _require(n == self.Shards)
        S = pitch if shard_size is None else shard_size
        _raise(load_library().ugo_fec_encode_host(self._h, shards.ctypes.data, G, S, pitch))

    def reconstruct_host(self, shards: np.ndarray, present: np.ndarray, shard_size: Optional[int] = None,
                         data_only=False, status: Optional[np.ndarray] = None) -> int:
        """Returns the aggregate status (0 or the first failing group's code);
        per-group codes go to `status` when given.  Does not raise for
        ErrTooFewShards groups (they are reported and left untouched)."""
        _require(shards.dtype == np.uint8 and shards.flags["C_CONTIGUOUS"] and shards.ndim == 3)
        G, n, pitch = shards.shape
        _require(n == self.Shards)
        present = np.ascontiguousarray(present, dtype=np.uint64)
        _require(present.size == G * self.mask_words)
        S = pitch if shard_size is None else shard_size
        st = None if status is None else status.ctypes.data
        if status is not None:
            _require(status.dtype == np.int8 and status.size == G)
        rc = load_library().ugo_fec_reconstruct_host(self._h, shards.ctypes.data, present.ctypes.data, G, S, pitch,
                                                     RECONSTRUCT_DATA_ONLY if data_only else 0, st)
        if rc not in (OK, ErrTooFewShards.code, ErrSingular.code):
            _raise(rc)
        return rc

    # ------------------------------------------- Go-shaped, one group per call
    def _stage(self, S: int) -> np.ndarray:
        """One pinned group [d+p][P] at the 16-B pitch P, reused across calls
        (the cgo shim's staging): the vector kernels, and the
        per-call service when it is on, serve it."""
        P = (S + 15) // 16 * 16
        need = self.Shards * P
        st = getattr(self, "_stage_buf", None)
        if st is None or st.size < need:
            if st is not None:
                host_free(st)
            st = self._stage_buf = host_alloc(max(need, self.Shards * 1488))
        return st[:need].reshape(1, self.Shards, P)

    def Encode(self, shards: List[bytearray]) -> None:
        """reedsolomon Encode: parity shards written in place (ugo/fec.go:238)."""
        if len(shards) != self.Shards:
            raise ErrTooFewShards(strerror(ErrTooFewShards.code))
        S = check_shards([len(s) for s in shards], nil_ok=False)
        buf = self._stage(S)
        for k in range(self.DataShards):
            buf[0, k, :S] = np.frombuffer(bytes(shards[k]), np.uint8)
        self.encode_host(buf, S)
        for k in range(self.DataShards, self.Shards):
            shards[k][:] = buf[0, k, :S].tobytes()

    def _reconstruct(self, shards: list, data_only: bool) -> None:
        if len(shards) != self.Shards:
            raise ErrTooFewShards(strerror(ErrTooFewShards.code))
        lens = [0 if s is None else len(s) for s in shards]
        S = check_shards(lens, nil_ok=True)
        mask = np.zeros(self.mask_words, np.uint64)
        buf = self._stage(S)
        for r, s in enumerate(shards):
            if lens[r]:
                mask[r >> 6] |= np.uint64(1 << (r & 63))
                buf[0, r, :S] = np.frombuffer(bytes(s), np.uint8)
        status = np.zeros(1, np.int8)
        rc = self.reconstruct_host(buf, mask, S, data_only, status)
        _raise(rc)
        limit = self.DataShards if data_only else self.Shards
        for r in range(limit):
            if not lens[r]:
                shards[r] = bytearray(buf[0, r, :S].tobytes())

    def Reconstruct(self, shards: list) -> None:
        """reedsolomon Reconstruct (ugo/fec.go:202): fills every missing shard."""
        self._reconstruct(shards, data_only=False)

    def ReconstructData(self, shards: list) -> None:
        self._reconstruct(shards, data_only=True)


def rc4_keystream(key: bytes, n: int) -> bytes:
    """RC4 keystream prefix (ugo/crypto.go's fixed-key per-packet cipher)."""
    out = (ctypes.c_uint8 * n)()
    k = (ctypes.c_uint8 * len(key)).from_buffer_copy(key)
    _raise(load_library().ugo_fec_rc4_keystream(ctypes.addressof(k), len(key), ctypes.addressof(out), n))
    return bytes(out)


def New(data_shards: int, parity_shards: int, device: int = 0) -> Encoder:
    """reedsolomon.New as called at ugo/fec.go:59."""
    return Encoder(data_shards, parity_shards, device)


def host_alloc(nbytes: int) -> np.ndarray:
    """Pinned host buffer (uint8 numpy view); free with host_free(arr)."""
    lib = load_library()
    p = ctypes.c_void_p()
    _raise(lib.ugo_fec_host_alloc(nbytes, ctypes.byref(p)))
    arr = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(nbytes,))
    return arr


def host_free(arr: np.ndarray) -> None:
    _raise(load_library().ugo_fec_host_free(ctypes.c_void_p(arr.ctypes.data)))


# ---------------------------------------------------------------- FEC object
UGO_FEC_MAX_PACKET = 1476
_CLOCK_T = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_void_p)


def _bind_conn(lib):
    if getattr(lib, "_conn_bound", False):
        return lib
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    lib.ugo_fecconn_new.argtypes = [i, i, i, i, ctypes.POINTER(vp)]
    lib.ugo_fecconn_free.argtypes = [vp]
    lib.ugo_fecconn_free.restype = None
    lib.ugo_fecconn_set_clock.argtypes = [vp, _CLOCK_T, vp]
    lib.ugo_fecconn_mark_data.argtypes = [vp, vp]
    lib.ugo_fecconn_mark_fec.argtypes = [vp, vp]
    lib.ugo_fecconn_get_next.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32)]
    lib.ugo_fecconn_set_next.argtypes = [vp, ctypes.c_uint32]
    lib.ugo_fecconn_input.argtypes = [vp, vp, sz, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint16),
                                      vp, sz, ctypes.POINTER(i), ctypes.POINTER(sz)]
    lib.ugo_fecconn_calc_ecc.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(sz), i, i, i]
    lib.ugo_fecconn_rx_len.argtypes = [vp, ctypes.POINTER(sz)]
    lib.ugo_fecconn_set_batch.argtypes = [vp, i, vp, sz, ctypes.POINTER(i), ctypes.POINTER(sz)]
    lib.ugo_fecconn_set_batch_ex.argtypes = [vp, i, ctypes.c_uint, vp, sz, ctypes.POINTER(i), ctypes.POINTER(sz)]
    lib.ugo_fecconn_flush.argtypes = [vp, vp, sz, ctypes.POINTER(i), ctypes.POINTER(sz)]
    lib.ugo_fecconn_pending.argtypes = [vp, ctypes.POINTER(sz)]
    lib.ugo_fecconn_service.argtypes = [vp, ctypes.c_int]
    lib._conn_bound = True
    return lib


class FecConn:
    """ugo's per-connection FEC object (ugo/fec.go:14-27) as implemented by the
    C++ host mirror (ugo_amd/csrc/host/fec.cpp) behind include/ugo_fec_conn.h."""

    def __init__(self, rxlimit: int, data_shards: int, parity_shards: int, device: int = 0):
        lib = _bind_conn(load_library())
        h = ctypes.c_void_p()
        _raise(lib.ugo_fecconn_new(rxlimit, data_shards, parity_shards, device, ctypes.byref(h)))
        self._h, self._lib = h, lib
        self.dataShards, self.parityShards = data_shards, parity_shards
        self._clock_cb = None
        self._out = (ctypes.c_uint8 * (data_shards * UGO_FEC_MAX_PACKET))()

    def close(self):
        if getattr(self, "_h", None):
            self._lib.ugo_fecconn_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_clock(self, fn):
        """fn() -> uint32 milliseconds (replaces currentMs, ugo/fec.go:73)."""
        self._clock_cb = _CLOCK_T(lambda _u: fn() & 0xFFFFFFFF)
        _raise(self._lib.ugo_fecconn_set_clock(self._h, self._clock_cb, None))

    def markData(self, buf: bytearray):
        c = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
        _raise(self._lib.ugo_fecconn_mark_data(self._h, ctypes.addressof(c)))

    def markFEC(self, buf: bytearray):
        c = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
        _raise(self._lib.ugo_fecconn_mark_fec(self._h, ctypes.addressof(c)))

    @property
    def next(self) -> int:
        v = ctypes.c_uint32()
        _raise(self._lib.ugo_fecconn_get_next(self._h, ctypes.byref(v)))
        return v.value

    @next.setter
    def next(self, v: int):
        _raise(self._lib.ugo_fecconn_set_next(self._h, v))

    def _recovered(self, nrec, rlen):
        if not nrec.value:
            return None
        raw = bytes(self._out)
        return [bytearray(raw[i * UGO_FEC_MAX_PACKET: i * UGO_FEC_MAX_PACKET + rlen.value])
                for i in range(nrec.value)]

    def input(self, wire: bytes):
        """decode + input (ugo/conn.go:394-396): returns (seqid, flag, recovered list | None)."""
        seq, flag = ctypes.c_uint32(), ctypes.c_uint16()
        nrec, rlen = ctypes.c_int(), ctypes.c_size_t()
        w = (ctypes.c_uint8 * len(wire)).from_buffer_copy(wire)
        _raise(self._lib.ugo_fecconn_input(self._h, ctypes.addressof(w), len(wire), ctypes.byref(seq),
                                           ctypes.byref(flag), ctypes.addressof(self._out), len(self._out),
                                           ctypes.byref(nrec), ctypes.byref(rlen)))
        return seq.value, flag.value, self._recovered(nrec, rlen)

    def set_batch(self, groups: int, overlap: bool = False):
        """Batched recovery (include/ugo_fec_conn.h): recoverable lossy groups are
        recovered `groups` at a time in one launch; 0 = per call.  overlap: the
        launch runs while input goes on, its shards come back one batch later
        (UGO_FECCONN_BATCH_OVERLAP).  Returns the recovered shards of groups that
        were pending (list | None)."""
        nrec, rlen = ctypes.c_int(), ctypes.c_size_t()
        need = max(groups, 1) * (2 if overlap else 1) * self.dataShards * UGO_FEC_MAX_PACKET
        new_out = (ctypes.c_uint8 * max(need, len(self._out)))()
        old_out, self._out = self._out, new_out
        try:
            _raise(self._lib.ugo_fecconn_set_batch_ex(self._h, groups, 1 if overlap else 0,
                                                      ctypes.addressof(self._out), len(self._out),
                                                      ctypes.byref(nrec), ctypes.byref(rlen)))
        except Exception:
            self._out = old_out
            raise
        rec = self._recovered(nrec, rlen)
        self._out = (ctypes.c_uint8 * need)()
        return rec

    def flush(self):
        """Recover every pending group now (list | None)."""
        nrec, rlen = ctypes.c_int(), ctypes.c_size_t()
        _raise(self._lib.ugo_fecconn_flush(self._h, ctypes.addressof(self._out), len(self._out),
                                           ctypes.byref(nrec), ctypes.byref(rlen)))
        return self._recovered(nrec, rlen)

    def service(self, idle_us: int = 0):
        """Per-call latency service on this object's encoder (ugo_fecconn_service);
        idle_us < 0 stops it."""
        _raise(self._lib.ugo_fecconn_service(self._h, idle_us))

    def pending(self) -> int:
        v = ctypes.c_size_t()
        _raise(self._lib.ugo_fecconn_pending(self._h, ctypes.byref(v)))
        return v.value

    def calcECC(self, data: List[bytearray], offset: int, maxlen: int):
        n = len(data)
        arrs = [(ctypes.c_uint8 * len(b)).from_buffer(b) for b in data]
        ptrs = (ctypes.c_void_p * n)(*[ctypes.addressof(a) for a in arrs])
        lens = (ctypes.c_size_t * n)(*[len(b) for b in data])
        _raise(self._lib.ugo_fecconn_calc_ecc(self._h, ptrs, lens, n, offset, maxlen))
        return data[self.dataShards:]

    def rx_len(self) -> int:
        v = ctypes.c_size_t()
        _raise(self._lib.ugo_fecconn_rx_len(self._h, ctypes.byref(v)))
        return v.value
