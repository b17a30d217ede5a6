#!/usr/bin/env python3
"""Where does ugo_fec_reconstruct_rows spend its time on small batches?

The FEC object's batched recovery reads lost groups' survivors in place, in
pinned pool buffers, through a pinned row-pointer table, pinned masks, into a
pinned output batch.  This probe times one launch (HIP events on the launch
stream, median of many) of a (10,3) x 1476-B data-only reconstruct for 1 and
64 groups with each of those four buffers in device memory or in pinned host
memory, and the staged-batch kernel (ugo_fec_reconstruct_into on a pinned
batch) beside it.  Prints one JSON line per case.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ugo_amd import fec  # noqa: E402

d, p, n, S, SP = 10, 3, 13, 1476, 1488


def timeit(fn, reps=200):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return round(t[len(t) // 2], 2), round(t[len(t) // 10], 2)


def main():
    enc = fec.New(d, p)
    keep = []

    def pinned(nbytes):
        a = fec.host_alloc(nbytes)
        keep.append(a)
        return a

    for G in (1, 64):
        rng = np.random.default_rng(G)
        nslots = 4096
        masks_np = np.full(G, (1 << n) - 1, np.uint64) & ~np.uint64(1 << 3)  # data row 3 lost
        slot = rng.permutation(nslots)[:G * n].reshape(G, n)
        for data_where in ("device", "pinned"):
            if data_where == "device":
                pool = torch.randint(0, 256, (nslots, SP), dtype=torch.uint8, device="cuda")
                base = pool.data_ptr()
            else:
                pool = pinned(nslots * SP).reshape(nslots, SP)
                pool[:] = rng.integers(0, 256, (nslots, SP), dtype=np.uint8)
                base = enc.device_address(pool.ctypes.data)
            rows_np = np.zeros((G, n), np.int64)
            for g in range(G):
                for r in range(n):
                    if (int(masks_np[g]) >> r) & 1:
                        rows_np[g, r] = base + int(slot[g, r]) * SP
            for table_where in ("device", "pinned"):
                if table_where == "device":
                    rows = torch.from_numpy(rows_np).cuda()
                    present = torch.from_numpy(masks_np.view(np.int64)).cuda()
                else:
                    rows = pinned(G * n * 8).view(np.int64).reshape(G, n)
                    rows[:] = rows_np
                    present = pinned(G * 8).view(np.uint64)
                    present[:] = masks_np
                for out_where in ("device", "pinned"):
                    if out_where == "device":
                        out = torch.zeros((p, G, SP), dtype=torch.uint8, device="cuda")
                    else:
                        out = torch.from_numpy(pinned(p * G * SP).reshape(p, G, SP))
                        # a CPU tensor aliasing pinned memory: pass its device address
                    if out_where == "pinned":
                        class _Out:  # data_ptr() = device address of the pinned buffer, shape/strides of out
                            def __init__(self, t):
                                self.t = t
                                self.shape = t.shape

                            def dim(self):
                                return 3

                            def is_contiguous(self):
                                return True

                            def element_size(self):
                                return 1

                            def data_ptr(self):
                                return enc.device_address(self.t.data_ptr())
                        o = _Out(out)
                    else:
                        o = out
                    med, p10 = timeit(lambda: enc.reconstruct_rows(rows, present, o, S, data_only=True))
                    print(json.dumps({"groups": G, "rows_data": data_where, "table_masks": table_where, "out": out_where,
                                      "median_us": med, "p10_us": p10}), flush=True)
        # the staged form for comparison: a pinned group-major batch, zero-copy reconstruct_into
        batch = pinned(G * n * SP).reshape(G, n, SP)
        batch[:] = rng.integers(0, 256, (G, n, SP), dtype=np.uint8)
        bt = torch.from_numpy(batch)
        present = torch.from_numpy(masks_np.view(np.int64)).cuda()
        out = torch.zeros((p, G, SP), dtype=torch.uint8, device="cuda")
        lib = fec.load_library()
        dev_batch = enc.device_address(batch.ctypes.data)

        def staged():
            fec._raise(lib.ugo_fec_reconstruct_into(enc._h, dev_batch, present.data_ptr(), G, S, SP, n * SP,
                                                    out.data_ptr(), G * SP, SP, 1, None,
                                                    torch.cuda.current_stream().cuda_stream))
        med, p10 = timeit(staged)
        print(json.dumps({"groups": G, "staged_batch_pinned_reconstruct_into": True, "median_us": med, "p10_us": p10}),
              flush=True)
        del bt
    for k in keep:
        fec.host_free(k)


if __name__ == "__main__":
    main()
