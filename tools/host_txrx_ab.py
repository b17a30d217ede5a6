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
    if "bind" in sys.argv[3:]:  # as bench.py's host_path: every thread on the GPU's node
        from ugo_amd import numa

        placement = numa.bind_to_node(numa.gpu_numa_node(0))
    d, p, S, slot = 10, 3, 1350, 1488
    G = int(os.environ.get("HAB_GROUPS", "65536"))
    n = d + p
    dev = torch.device("cuda:0")
    # HAB_DUMMY=k: k streams that each issue one host->device copy before the library creates its
    # own (the copy engine a stream gets depends on what the process did before, profiles/r5/txgraph*)
    dummies = []
    for _ in range(int(os.environ.get("HAB_DUMMY", "0"))):
        st = torch.cuda.Stream(dev)
        with torch.cuda.stream(st):
            torch.empty(4096, dtype=torch.uint8).pin_memory().to(dev, non_blocking=True)
        st.synchronize()
        dummies.append(st)
    enc = fec.Encoder(d, p, device=0)
    if os.environ.get("HAB_COPYQ"):  # 1: the low-priority copy stream (ugo_fec_set_host_copy_queue)
        enc.set_host_copy_queue(os.environ["HAB_COPYQ"] == "1")
    if os.environ.get("HAB_ROUTE"):  # copy / mapped: tx_assemble_host's wire route (default copy)
        enc.set_tx_host_route(os.environ["HAB_ROUTE"])
    gen = torch.Generator(device=dev).manual_seed(11)
    padb = fec.rc4_keystream(b"1234567890123456", slot)
    if "rxfirst" in sys.argv[3:]:  # as bench.py: the host RX case first, on the same context
        seq = torch.arange(G * n, device=dev, dtype=torch.int64)
        seq = seq[torch.rand(G * n, device=dev, generator=gen) >= 0.05]
        npk = seq.numel()
        w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
        hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
        for b in range(4):
            hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
        hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
        w[:, :6] = hdr ^ torch.frombuffer(bytearray(padb[:6]), dtype=torch.uint8).to(dev)
        ring = fec.host_alloc(npk * slot).reshape(npk, slot)
        rl = fec.host_alloc(npk * 2).view(np.uint16)
        out = fec.host_alloc(G * p * 1360).reshape(G * p, 1360)
        torch.from_numpy(ring).copy_(w)
        rl[:] = 1476
        del w
        rx = []
        for _ in range(7):
            t0 = time.perf_counter()
            enc.rx_recover_host(ring, rl, S, G, pad=padb, out=out, max_out=G)
            rx.append((time.perf_counter() - t0) * 1e3)
        for b in (ring, rl.view(np.uint8), out):
            fec.host_free(b)
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
        time.sleep(float(os.environ.get("HAB_GAP_MS", "0")) / 1e3)  # separates the calls in a trace
    digest = hashlib.sha1(wire[:, :1476].tobytes() + wl.tobytes()).hexdigest()[:16]
    for b in (pk, ln.view(np.uint8), wire, wl.view(np.uint8)):
        fec.host_free(b)
    tx_ms = sorted(tx)[len(tx) // 2]
    print(json.dumps({"label": label, "groups": G, "dummy_streams": len(dummies), "placement": placement,
                      "tx_ms": round(tx_ms, 3),
                      "tx_pcie_GBps": round(G * (d + n) * slot / tx_ms / 1e6, 2), "tx_all_ms": [round(t, 2) for t in tx],
                      "tx_digest": digest,
                      "rx_all_ms": [round(t, 2) for t in rx] if "rxfirst" in sys.argv[3:] else None}))


if __name__ == "__main__":
    main()
