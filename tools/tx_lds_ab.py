"""Device-resident tx_assemble timed like bench.py's rx_tx.tx case (65,536
(10+3) groups of 10 full 1476-B packets, 1488-B slots, RC4, 2 cold copies of
every buffer alternating), for A/B runs of library builds (UGO_FEC_LIB), with
a digest of every wire packet's bytes [0, wire_len) to compare builds.  Not
product code.

  python3 tools/tx_lds_ab.py LABEL [rounds] [reps] [max_len]
"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import numpy as np
    import torch

    from ugo_amd import fec

    label = sys.argv[1] if len(sys.argv) > 1 else "?"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    max_len = int(sys.argv[4]) if len(sys.argv) > 4 else 1476
    d, p, n, G = 10, 3, 13, 65536
    slot = (max_len + 15) // 16 * 16
    dev = torch.device("cuda:0")
    enc = fec.New(d, p)
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", slot)), dtype=torch.uint8).to(dev)
    gen = torch.Generator(device=dev).manual_seed(0x7C)
    pks = [torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device=dev, generator=gen) for _ in range(2)]
    if os.environ.get("TXAB_MIXED"):  # mixed lengths 6..max_len
        tl = torch.randint(6, max_len + 1, (G * d,), dtype=torch.int32, device=dev, generator=gen).to(torch.int16)
    else:
        tl = torch.full((G * d,), max_len, dtype=torch.int16, device=dev)
    wires = [torch.empty((G * n, slot), dtype=torch.uint8, device=dev) for _ in range(2)]
    wls = [torch.empty(G * n, dtype=torch.int16, device=dev) for _ in range(2)]
    kid = fec.KERNEL_IDS["tx_assemble"]

    def tx(r):
        i = r % 2
        enc.tx_assemble(pks[i], tl, wires[i], wls[i], pad=pad, max_len=max_len)

    for r in range(4):
        tx(r)
    torch.cuda.synchronize()
    wl = wls[0].to(torch.int32)
    keep = torch.arange(slot, device=dev)[None, :] < wl[:, None]
    dig = hashlib.sha256(wires[0][keep].cpu().numpy().tobytes() + wls[0].cpu().numpy().tobytes()).hexdigest()[:16]
    tx_bytes = int(tl.to(torch.int64).sum()) + int(wl.to(torch.int64).sum())
    out = {"label": label, "digest": dig, "ms": []}
    for _ in range(rounds):
        enc.timing_begin(4 * reps)
        for r in range(reps):
            tx(r)
        recs, _ = enc.timing_end()
        out["ms"].append(round(float(recs["ms"][recs["kernel"] == kid].sum()) / reps, 4))
    ms = sorted(out["ms"])[len(out["ms"]) // 2]
    out["tx_ms"] = ms
    out["tx_frac"] = round(tx_bytes / (ms * 1e-3) / 8e12, 4)
    print(json.dumps(out), flush=True)
    enc.close()


if __name__ == "__main__":
    main()
