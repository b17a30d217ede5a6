"""Timeline of one ugo_fec_tx_assemble_host call (the bench's tx_host case:
65,536 (10+3) groups of 1476-B packets in 1488-B slots, RC4 pad, pinned
buffers) for rocprofv3 --kernel-trace --memory-copy-trace: where the call's
time goes between the H2D copies, the assembly kernels and the D2H copies.
HTT_ROUTE=copy|mapped selects the wire route (default copy).  Not product code.

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/htx -o run \
      -- python3 tools/host_tx_trace.py
  python3 tools/host_rx_trace.py --summarise gpurun_out/htx
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(reps=10):
    import numpy as np
    import torch

    from ugo_amd import fec

    d, p, G, slot = 10, 3, int(os.environ.get("HTT_GROUPS", "65536")), 1488
    n = d + p
    dev = torch.device("cuda:0")
    # HTT_DUMMY=k: k torch streams each make one small host->device copy before the library
    # creates its streams (as tools/host_txrx_ab.py HAB_DUMMY)
    dummies = []
    for _ in range(int(os.environ.get("HTT_DUMMY", "0"))):
        st = torch.cuda.Stream(dev)
        with torch.cuda.stream(st):
            torch.empty(4096, dtype=torch.uint8).pin_memory().to(dev, non_blocking=True)
        st.synchronize()
        dummies.append(st)
    enc = fec.Encoder(d, p, device=0)
    enc.set_tx_host_route(os.environ.get("HTT_ROUTE", "copy"))
    gen = torch.Generator(device=dev).manual_seed(9)
    padb = fec.rc4_keystream(b"1234567890123456", slot)
    pk = fec.host_alloc(G * d * slot).reshape(G * d, slot)
    ln = fec.host_alloc(G * d * 2).view(np.uint16)
    wire = fec.host_alloc(G * n * slot).reshape(G * n, slot)
    wl = fec.host_alloc(G * n * 2).view(np.uint16)
    torch.from_numpy(pk).copy_(torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device=dev, generator=gen))
    ln[:] = 1476
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        enc.tx_assemble_host(pk, ln, wire, wl, pad=padb, max_len=1476)
        times.append((time.perf_counter() - t0) * 1e3)
        time.sleep(0.01)  # a gap that separates the calls in the trace
    print(json.dumps({"groups": G, "call_ms": [round(t, 3) for t in times],
                      "bytes_in": G * d * slot, "bytes_out": G * n * slot}))
    for b in (pk, ln.view(np.uint8), wire, wl.view(np.uint8)):
        fec.host_free(b)


if __name__ == "__main__":
    run()
