"""RX placement time against how the batch storage was allocated (round 6).

The frame-row placement of the bench's ring ran 0.407-0.454 ms in order on
one box depending only on which allocation backed the batch
(profiles/r6/rx_frames/same_storage_ab.jsonl).  Here the two rings stay fixed
for the whole run and only the batch storage changes: per trial, batch pairs
from torch's allocator, from hipMalloc and from hipExtMallocWithFlags(
hipDeviceMallocContiguous), each timed in alternating rounds (frame rows and
payload rows on the same storage).  Is the spread the batch's, and does a
physically contiguous batch always land in the fast mode?

Usage: python tools/rx_alloc_ab.py [trials] [reps]  (one JSON line per trial)
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


def main(trials=6, reps=12, rounds=3, mode="kinds"):
    import torch

    from ugo_amd import fec

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]

    d, p, n, S, slot = 10, 3, 13, 1470, 1488
    G = 65536
    span = n * G * 1536
    dev = torch.device("cuda:0")
    enc = fec.New(d, p)
    lib = fec.load_library()
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", slot)), dtype=torch.uint8).to(dev)
    gen = torch.Generator(device=dev).manual_seed(0x79)
    rx_id = fec.KERNEL_IDS["rx_assemble"]
    seq = torch.arange(G * n, device=dev, dtype=torch.int64)
    seq = seq[torch.rand(G * n, device=dev, generator=gen) >= 0.05]
    npk = seq.numel()
    lens = torch.full((npk,), 1476, dtype=torch.int16, device=dev)
    rx_bytes = npk * (1476 + S)
    rings = []
    for _ in range(2):
        w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
        hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
        for b in range(4):
            hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
        hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
        w[:, :6] = hdr ^ pad[:6]
        rings.append(w)
    pres = [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(2)]
    stream = torch.cuda.current_stream().cuda_stream

    def hip_alloc(nbytes, flags=None):
        ptr = ctypes.c_void_p()
        st = hip.hipMalloc(ctypes.byref(ptr), nbytes) if flags is None else hip.hipExtMallocWithFlags(
            ctypes.byref(ptr), nbytes, flags)
        if st != 0:
            raise RuntimeError(f"hip allocation of {nbytes} B failed: {st}")
        return ptr.value

    def time_layout(ptrs, frames, per_copy=False):
        pitch = 1536 if frames else 1472
        entry = lib.ugo_fec_rx_assemble_frames if frames else lib.ugo_fec_rx_assemble

        def rx(r):
            i = r % 2
            pres[i].zero_()
            st = entry(enc._h, rings[i].data_ptr(), slot, lens.data_ptr(), npk, pad.data_ptr(), 0, G, ptrs[i], S,
                       G * pitch, pitch, pres[i].data_ptr(), None, stream)
            if st != 0:
                raise RuntimeError(f"rx_assemble status {st}")

        for r in range(2):
            rx(r)
        enc.timing_begin(16 * reps)
        for r in range(reps):
            rx(r)
        recs, _ = enc.timing_end()
        ms = recs["ms"][recs["kernel"] == rx_id]
        if per_copy:  # launches per call are equal: split the calls by copy
            per = ms.reshape(reps, -1).sum(axis=1)
            return [float(per[0::2].mean()), float(per[1::2].mean())]
        return float(ms.sum()) / reps

    def time_ring(rps, ptrs):
        pitch = 1536

        def rx(r):
            i = r % 2
            pres[i].zero_()
            st = lib.ugo_fec_rx_assemble_frames(enc._h, rps[i], slot, lens.data_ptr(), npk, pad.data_ptr(), 0, G,
                                                ptrs[i], S, G * pitch, pitch, pres[i].data_ptr(), None, stream)
            if st != 0:
                raise RuntimeError(f"rx_assemble status {st}")

        for r in range(2):
            rx(r)
        enc.timing_begin(16 * reps)
        for r in range(reps):
            rx(r)
        recs, _ = enc.timing_end()
        per = recs["ms"][recs["kernel"] == rx_id].reshape(reps, -1).sum(axis=1)
        return [float(per[0::2].mean()), float(per[1::2].mean())]

    if mode == "offset":
        # one allocation per copy, the batch placed at offsets into it: the same physical pages,
        # shifted against the batch's planes
        slack = 384 << 20
        bases = [hip_alloc(span + slack) for _ in range(2)]
        offs = [0, 2, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 320]
        for rnd in range(rounds):
            for o in (offs if rnd % 2 == 0 else offs[::-1]):
                t = time_layout([b + (o << 20) for b in bases], True, per_copy=True)
                print(json.dumps({"round": rnd, "offset_MiB": o, "bases": [hex(b) for b in bases],
                                  "frames_ms_per_copy": [round(x, 4) for x in t]}), flush=True)
        for b in bases:
            hip.hipFree(b)
        enc.close()
        return

    if mode == "ring":
        # the batch pair fixed, the rings re-allocated per trial (contents copied from the first rings):
        # does the placement mode follow the ring's pages as well as the batch's?
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        bats = [hip_alloc(span) for _ in range(2)]
        src = [r for r in rings]
        rb = npk * slot
        for t in range(trials):
            dummy = hip_alloc((1 + 53 * t) << 20)
            rp = [hip_alloc(rb) for _ in range(2)]
            for i in range(2):
                hip.hipMemcpy(rp[i], src[i].data_ptr(), rb, 3)
            torch.cuda.synchronize()
            ms = time_ring(rp, bats)
            print(json.dumps({"trial": t, "rings": [hex(x) for x in rp], "bats": [hex(x) for x in bats],
                              "frames_ms_per_copy": [round(x, 4) for x in ms]}), flush=True)
            for x in rp:
                hip.hipFree(x)
            hip.hipFree(dummy)
        enc.close()
        return

    if mode == "pmc":
        # hipMalloc pairs after dummies of varying size, frame rows timed per copy: a short run for
        # rocprofv3 --pmc passes (dispatch order: per trial 2 + reps placing launches, copies 0, 1, ...)
        for t in range(trials):
            dummy = hip_alloc((1 + 53 * t) << 20)
            ptrs = [hip_alloc(span) for _ in range(2)]
            ms = time_layout(ptrs, True, per_copy=True)
            print(json.dumps({"trial": t, "ptr": [hex(x) for x in ptrs], "frames_ms_per_copy": [round(x, 4) for x in ms]}),
                  flush=True)
            for x in ptrs:
                hip.hipFree(x)
            hip.hipFree(dummy)
        enc.close()
        return

    check = None
    for t in range(trials):
        dummy = hip_alloc((1 + 53 * t) << 20)  # shift where the next allocations land
        kinds = {}
        keep = []
        tt = [torch.empty(span, dtype=torch.uint8, device=dev) for _ in range(2)]
        keep.append(tt)
        kinds["torch"] = [x.data_ptr() for x in tt]
        kinds["hipMalloc"] = [hip_alloc(span) for _ in range(2)]
        kinds["contiguous"] = [hip_alloc(span, HIP_DEVICE_MALLOC_CONTIGUOUS) for _ in range(2)]
        times = {k: {"frames": [], "payload": []} for k in kinds}
        names = list(kinds)
        for rnd in range(rounds):
            order = names[rnd % len(names):] + names[:rnd % len(names)]
            for k in order:
                for lay in (("frames", "payload") if rnd % 2 == 0 else ("payload", "frames")):
                    times[k][lay].append(time_layout(kinds[k], lay == "frames"))
        # the placed rows are the same bytes whatever backs them (first trial: contiguous vs torch)
        if check is None:
            time_layout(kinds["contiguous"], True)
            torch.cuda.synchronize()
            a = torch.empty(span, dtype=torch.uint8, device=dev)
            hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            torch.cuda.synchronize()
            hip.hipMemcpy(a.data_ptr(), kinds["contiguous"][0], span, 3)
            time_layout([tt[0].data_ptr(), tt[1].data_ptr()], True)
            torch.cuda.synchronize()
            v = a[:n * G * 1536].view(n, G, 1536)[:, :, :1476]
            w = tt[0][:n * G * 1536].view(n, G, 1536)[:, :, :1476]
            pm = pres[0].clone()
            got = ((pm[None, :] >> torch.arange(n, device=dev)[:, None]) & 1).bool()
            check = bool(torch.equal(v[got], w[got]))
            del a, v, w
        line = {"trial": t, "check_contiguous_eq_torch": check,
                "ptr": {k: [hex(x) for x in v] for k, v in kinds.items()}, "dummy": hex(dummy),
                "rings": [hex(r.data_ptr()) for r in rings]}
        for k in kinds:
            line[k] = {lay: {"ms": round(statistics.median(v), 4),
                             "frac": round(rx_bytes / (statistics.median(v) * 1e-3) / 8e12, 4),
                             "rounds": [round(x, 4) for x in v]} for lay, v in times[k].items()}
        print(json.dumps(line), flush=True)
        for k in ("hipMalloc", "contiguous"):
            for x in kinds[k]:
                hip.hipFree(x)
        hip.hipFree(dummy)
        del keep, tt
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    enc.close()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "ring":
        main(trials=int(sys.argv[2]), reps=int(sys.argv[3]), mode="ring")
    elif len(sys.argv) > 1 and sys.argv[1] == "pmc":
        main(trials=int(sys.argv[2]), reps=int(sys.argv[3]), mode="pmc")
    elif len(sys.argv) > 1 and sys.argv[1] == "offset":
        main(reps=int(sys.argv[2]) if len(sys.argv) > 2 else 12, rounds=2, mode="offset")
    else:
        main(*(int(a) for a in sys.argv[1:3]))
