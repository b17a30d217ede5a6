"""Host-memory TX and RX calls timed back to back (the bench's host_path
shapes: 65,536 (10+3) groups, 1488-B slots, RC4 pad, pinned buffers), for A/B
runs of library builds (UGO_FEC_LIB selects one, tools/build_variant.sh makes
them).  Prints one JSON line: median ms of tx_assemble_host and
rx_recover_host, and a digest of the TX output for comparing builds.  Not
product code.

  python3 tools/host_txrx_ab.py LABEL [reps]
"""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import numpy as np
    import torch

    from ugo_amd import fec

    label = sys.argv[1] if len(sys.argv) > 1 else "?"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    placement = None
    if len(sys.argv) > 3 and sys.argv[3] == "bind":  # as bench.py's host_path: every thread on the GPU's node
        from ugo_amd import numa

        placement = numa.bind_to_node(numa.gpu_numa_node(0))
    d, p, S, G, slot = 10, 3, 1350, 65536, 1488
    n = d + p
    dev = torch.device("cuda:0")
    enc = fec.Encoder(d, p, device=0)
    gen = torch.Generator(device=dev).manual_seed(11)
    padb = fec.rc4_keystream(b"1234567890123456", slot)
    pk = fec.host_alloc(G * d * slot).reshape(G * d, slot)
    ln = fec.host_alloc(G * d * 2).view(np.uint16)
    wire = fec.host_alloc(G * n * slot).reshape(G * n, slot)
    wl = fec.host_alloc(G * n * 2).view(np.uint16)
    torch.from_numpy(pk).copy_(torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device=dev, generator=gen))
    ln[:] = 1476
    tx = []
    for _ in range(reps):
        t0 = time.perf_counter()
        enc.tx_assemble_host(pk, ln, wire, wl, pad=padb, max_len=1476)
        tx.append((time.perf_counter() - t0) * 1e3)
    digest = hashlib.sha1(wire[:, :1476].tobytes() + wl.tobytes()).hexdigest()[:16]
    for b in (pk, ln.view(np.uint8), wire, wl.view(np.uint8)):
        fec.host_free(b)
    tx_ms = sorted(tx)[len(tx) // 2]
    print(json.dumps({"label": label, "placement": placement, "tx_ms": round(tx_ms, 3),
                      "tx_pcie_GBps": round(G * (d + n) * slot / tx_ms / 1e6, 2), "tx_all_ms": [round(t, 2) for t in tx],
                      "tx_digest": digest}))


if __name__ == "__main__":
    main()
