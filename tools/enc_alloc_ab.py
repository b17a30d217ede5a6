"""Headline encode time against the batch's allocation (round 6).

RX placement runs in a fast or a slow mode set by the physical pages behind
its batch (tools/rx_alloc_ab.py).  Does the headline encode
(65,536 groups of (10+3) x 1350 B, planar [13][G][1360]) do the same?  Per
trial a pair of batches from hipMalloc after a dummy allocation of varying
size, the encode timed per copy with hipExtLaunchKernel events.

Usage: python tools/enc_alloc_ab.py [trials] [reps]  (one JSON line per trial)
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(trials=10, reps=20, mode="pairs", flags=0):
    import torch

    from ugo_amd import fec

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]

    d, p, n, S, pitch, G = 10, 3, 13, 1350, 1360, 65536
    span = n * G * pitch
    algo = n * S * G  # algorithmic bytes per launch
    enc = fec.New(d, p)
    lib = fec.load_library()
    eid = fec.KERNEL_IDS["encode"]
    stream = torch.cuda.current_stream().cuda_stream

    def alloc(nbytes):
        ptr = ctypes.c_void_p()
        if hip.hipMalloc(ctypes.byref(ptr), nbytes) != 0:
            raise RuntimeError("hipMalloc failed")
        return ptr.value

    def time_pair(ptrs):
        def run(r):
            st = lib.ugo_fec_encode_strided(enc._h, ptrs[r % 2], G, S, G * pitch, pitch, stream)
            if st != 0:
                raise RuntimeError(f"encode status {st}")

        for r in range(4):
            run(r)
        enc.timing_begin(4 * reps)
        for r in range(reps):
            run(r)
        recs, _ = enc.timing_end()
        ms = recs["ms"][recs["kernel"] == eid].reshape(reps, -1).sum(axis=1)
        return [float(ms[0::2].mean()), float(ms[1::2].mean())]

    if mode == "carve":
        # one large hipMalloc region per trial; the pair carved at 1-GiB-aligned virtual addresses
        # inside it and at 2-MiB-aligned ones off those boundaries (same region, same pages pool)
        hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        GiB = 1 << 30
        for t in range(trials):
            dummy = alloc((1 + 53 * t) << 20)
            region = 14 * GiB
            if flags:
                ptr = ctypes.c_void_p()
                if hip.hipExtMallocWithFlags(ctypes.byref(ptr), region, flags) != 0:
                    raise RuntimeError("hipExtMallocWithFlags failed")
                base = ptr.value
            else:
                base = alloc(region)
            a0 = (base + GiB - 1) // GiB * GiB
            line = {"trial": t, "base": hex(base), "flags": flags}
            for name, pair in (("aligned_1G", [a0, a0 + 2 * GiB]), ("off_258M", [a0 + 4 * GiB + (258 << 20), a0 + 6 * GiB + (258 << 20)]),
                               ("aligned_1G_b", [a0 + 8 * GiB, a0 + 10 * GiB])):
                for x in pair:
                    hip.hipMemset(x, 0x5A, span)
                per = time_pair(pair)
                line[name] = {"ms": [round(x, 5) for x in per], "frac": [round(algo / (x * 1e-3) / 8e12, 4) for x in per]}
            print(json.dumps(line), flush=True)
            hip.hipFree(base)
            hip.hipFree(dummy)
        enc.close()
        return

    def alloc_flags(nbytes, fl):
        hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        ptr = ctypes.c_void_p()
        if hip.hipExtMallocWithFlags(ctypes.byref(ptr), nbytes, fl) != 0:
            raise RuntimeError("hipExtMallocWithFlags failed")
        return ptr.value

    for t in range(trials):
        dummy = alloc((1 + 53 * t) << 20)
        ptrs = [alloc(span) if not flags else alloc_flags(span, flags) for _ in range(2)]
        for x in ptrs:
            hip.hipMemset(x, 0x5A, span)

        def run(r):
            st = lib.ugo_fec_encode_strided(enc._h, ptrs[r % 2], G, S, G * pitch, pitch, stream)
            if st != 0:
                raise RuntimeError(f"encode status {st}")

        for r in range(4):
            run(r)
        enc.timing_begin(4 * reps)
        for r in range(reps):
            run(r)
        recs, _ = enc.timing_end()
        ms = recs["ms"][recs["kernel"] == eid].reshape(reps, -1).sum(axis=1)
        per = [float(ms[0::2].mean()), float(ms[1::2].mean())]
        print(json.dumps({"trial": t, "ptr": [hex(x) for x in ptrs], "encode_ms_per_copy": [round(x, 5) for x in per],
                          "frac_per_copy": [round(algo / (x * 1e-3) / 8e12, 4) for x in per]}), flush=True)
        for x in ptrs:
            hip.hipFree(x)
        hip.hipFree(dummy)
    enc.close()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] in ("carve", "contig"):
        main(trials=int(sys.argv[2]), reps=int(sys.argv[3]), mode=sys.argv[1] if sys.argv[1] == "carve" else "pairs",
             flags=int(sys.argv[4]) if len(sys.argv) > 4 else (4 if sys.argv[1] == "contig" else 0))
    else:
        main(*(int(a) for a in sys.argv[1:3]))
