"""Timeline of one ugo_fec_rx_recover_host call (the bench's rx_host case:
65,536 (10+3)x1350 groups, 5% loss, rc4 pad, pinned ring) for rocprofv3
--kernel-trace --memory-copy-trace: where the call's time goes between the
H2D stages, the assembly kernels, the recovery and the D2H.  Not product code.

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hrx -o run \
      -- python3 tools/host_rx_trace.py
  python3 tools/host_rx_trace.py --summarise gpurun_out/hrx
"""
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(reps=10):
    import numpy as np
    import torch

    from ugo_amd import fec

    d, p, S, G, slot = 10, 3, 1350, 65536, 1488
    n = d + p
    dev = torch.device("cuda:0")
    enc = fec.Encoder(d, p, device=0)
    gen = torch.Generator(device=dev).manual_seed(5)
    pad = torch.randint(0, 256, (slot,), dtype=torch.uint8, device=dev, generator=gen)
    seq = torch.arange(G * n, device=dev, dtype=torch.int64)
    seq = seq[torch.rand(G * n, device=dev, generator=gen) >= 0.05]
    npk = seq.numel()
    w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
    hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
    for b in range(4):
        hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
    hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
    w[:, :6] = hdr ^ pad[:6]
    ring = fec.host_alloc(npk * slot).reshape(npk, slot)
    lens = fec.host_alloc(npk * 2).view(np.uint16)
    out = fec.host_alloc(G * p * 1360).reshape(G * p, 1360)
    torch.from_numpy(ring).copy_(w)
    lens[:] = 1476
    padb = pad.cpu().numpy().tobytes()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = enc.rx_recover_host(ring, lens, S, G, pad=padb, out=out, max_out=G)
        times.append((time.perf_counter() - t0) * 1e3)
        time.sleep(0.01)  # a gap that separates the calls in the trace
    print(json.dumps({"npk": npk, "lossy": r[0], "call_ms": [round(t, 3) for t in times],
                      "ring_bytes": npk * slot}))
    for b in (ring, lens.view(np.uint8), out):
        fec.host_free(b)


def summarise(d):
    import csv

    ev = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append(("K " + r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0))
    for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            nb = int(r.get("Bytes") or r.get("Size") or 0)
            ev.append(("C " + r.get("Direction", r.get("Operation", "?")), int(r["Start_Timestamp"]),
                       int(r["End_Timestamp"]), nb))
    ev.sort(key=lambda e: e[1])
    # the last call: the events after the last gap of > 3 ms (the driver sleeps 10 ms between calls)
    cut, end = 0, 0
    for i, e in enumerate(ev):
        if i and e[1] - end > 3_000_000:
            cut = i
        end = max(end, e[2])
    last = ev[cut:]
    t0 = last[0][1]
    agg = {}
    for name, s, e, nb in last:
        a = agg.setdefault(name, [0, 0, 0, 1e30, 0])
        a[0] += 1
        a[1] += e - s
        a[2] += nb
        a[3] = min(a[3], s - t0)
        a[4] = max(a[4], e - t0)
    span = max(e for _, _, e, _ in last) - t0
    print(json.dumps({"call_span_ms": span / 1e6, "events": len(last)}))
    for name, (cnt, busy, nb, first, lastend) in sorted(agg.items(), key=lambda x: x[1][3]):
        print(json.dumps({"what": name, "count": cnt, "busy_ms": round(busy / 1e6, 3), "bytes": nb,
                          "GBps_busy": round(nb / busy, 2) if busy and nb else None,
                          "first_start_ms": round(first / 1e6, 3), "last_end_ms": round(lastend / 1e6, 3)}))
    # copy-engine occupancy: union of H2D intervals
    for kind in sorted({n for n, *_ in last if n.startswith("C ")}):
        iv = sorted((s, e) for n, s, e, _ in last if n == kind)
        tot, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        print(json.dumps({"union_busy": kind, "ms": round(tot / 1e6, 3)}))


def per_call(d):
    """Every call of the trace (split at the 10-ms gaps run() leaves): span,
    H2D busy / union / first-start / last-end, the gaps between consecutive H2D
    copies, and the tail after the last H2D (recovery + D2H)."""
    import csv

    ev = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append(("K", r["Kernel_Name"][:30], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0))
    for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            nb = int(r.get("Bytes") or r.get("Size") or 0)
            ev.append(("C", r.get("Direction", r.get("Operation", "?")), int(r["Start_Timestamp"]),
                       int(r["End_Timestamp"]), nb))
    ev.sort(key=lambda e: e[2])
    calls, cur, end = [], [], 0
    for e in ev:
        if cur and e[2] - end > 3_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = max(end, e[3])
    calls.append(cur)
    for k, c in enumerate(calls):
        t0 = c[0][2]
        h2d = sorted((s, e, nb) for kind, what, s, e, nb in c if kind == "C" and "HOST_TO_DEVICE" in what.upper()
                     and e - s > 200_000)  # the ring copies (the trace carries no sizes): > 0.2 ms each
        d2h = [(s, e, nb) for kind, what, s, e, nb in c if kind == "C" and "DEVICE_TO_HOST" in what.upper()]
        gaps = [round((h2d[i + 1][0] - h2d[i][1]) / 1e3, 1) for i in range(len(h2d) - 1)]
        span = max(e for *_, s, e, nb in c) - t0
        rates = [round((e - s) / 1e6, 3) for s, e, nb in h2d]
        print(json.dumps({
            "call": k, "span_ms": round(span / 1e6, 3), "events": len(c),
            "to_first_h2d_ms": round((h2d[0][0] - t0) / 1e6, 3) if h2d else None,
            "h2d_n": len(h2d), "h2d_busy_ms": round(sum(e - s for s, e, _ in h2d) / 1e6, 3),
            "h2d_ms": rates, "h2d_gaps_us": gaps,
            "last_h2d_end_ms": round((h2d[-1][1] - t0) / 1e6, 3) if h2d else None,
            "d2h_busy_ms": round(sum(e - s for s, e, _ in d2h) / 1e6, 3),
            "tail_after_last_h2d_ms": round((t0 + span - h2d[-1][1]) / 1e6, 3) if h2d else None,
            "kernel_busy_ms": round(sum(e - s for kind, _, s, e, _ in c if kind == "K") / 1e6, 3)}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--calls":
        per_call(sys.argv[2])
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[1] == "--summarise":
        summarise(sys.argv[2])
    else:
        run()
