"""bench.py's service_interference leg on its own (a resident per-call service
block against the bench step and a pinned-host encode on the same GPU), for
A/B runs of library builds (UGO_FEC_LIB).  SVI_TX=1: one host TX call first, on
a context left open through the samples (SVI_COPYQ=1: with the low-priority
copy queue on that context); the line carries the process's KFD queues; SVI_EXTRA=k,prio: k more torch
streams of that priority alive through the samples.  Prints one JSON line.  Not product
code.

  python3 tools/svc_interference.py LABEL
"""
import json
import os
import sys
import types

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import numpy as np

    import bench
    from ugo_amd import fec

    label = sys.argv[1] if len(sys.argv) > 1 else "?"
    args = types.SimpleNamespace(seed=0x5EED)
    enc = fec.New(10, 3, device=0)
    raw = fec.host_alloc(64 * 13 * 1472)
    keep = []
    # SVI_EXTRA=k,prio: k torch streams of that priority (0 normal, -1 high), each used once, alive
    # through the samples (more hardware queues in the process)
    extra = []
    if os.environ.get("SVI_EXTRA"):
        import torch

        k, prio = (int(x) for x in os.environ["SVI_EXTRA"].split(","))
        for _ in range(k):
            st = torch.cuda.Stream(device=0, priority=prio)
            with torch.cuda.stream(st):
                torch.ones(1024, device="cuda").sum()
            st.synchronize()
            extra.append(st)
    if os.environ.get("SVI_TX"):  # a host TX call first, on a context that stays open (as an application's)
        G, d, n, slot = 4096, 10, 13, 1488
        tx = fec.New(d, 3, device=0)
        pk = fec.host_alloc(G * d * slot).reshape(G * d, slot)
        ln = fec.host_alloc(G * d * 2).view(np.uint16)
        wire = fec.host_alloc(G * n * slot).reshape(G * n, slot)
        wl = fec.host_alloc(G * n * 2).view(np.uint16)
        pk[:] = 1
        ln[:] = 1476
        if os.environ.get("SVI_COPYQ"):  # the opt-in low-priority H2D stream on that context
            tx.set_host_copy_queue(True)
        tx.tx_assemble_host(pk, ln, wire, wl, max_len=1476)
        keep = [tx, pk, ln, wire, wl]
    try:
        res = bench.service_interference(args, 0, enc, raw)
    finally:
        fec.host_free(raw)
        enc.close()
        if keep:
            for b in keep[1:]:
                fec.host_free(b.reshape(-1).view(np.uint8))
            keep[0].close()
    res["label"] = label
    res["hsa_queues"] = kfd_queues()
    res["gpu_max_hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
    print(json.dumps(res))


def kfd_queues():
    """The process's KFD user queues (/sys/class/kfd/kfd/proc/<pid>/queues), each
    with whatever attributes the node exposes; None where the node is absent."""
    base = f"/sys/class/kfd/kfd/proc/{os.getpid()}/queues"
    if not os.path.isdir(base):
        return None
    out = []
    for q in sorted(os.listdir(base), key=lambda x: int(x) if x.isdigit() else 0):
        attrs = {}
        for a in sorted(os.listdir(os.path.join(base, q))):
            try:
                attrs[a] = open(os.path.join(base, q, a)).read().strip()[:40]
            except OSError as ex:
                attrs[a] = f"<{ex.errno}>"
        out.append({"id": q, **attrs})
    return out


if __name__ == "__main__":
    main()
