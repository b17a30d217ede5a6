"""A/B of the RX placement layouts on one box, interleaved:
payload rows (ugo_fec_rx_assemble: realigned payload at column 0) against
frame rows (ugo_fec_rx_assemble_frames: the decrypted packet, payload at
column 6, no realignment), each followed by the lossy list + list
reconstruct of the data-only recovery on its own layout.  The bench's rx_tx
ring: 65,536 (10+3) groups, 5 % uniform loss, 1476-B packets in 1488-B slots,
RC4, in order and shuffled, cold (2 copies of every buffer alternate).
Checks first that the two layouts agree (presence, payload columns, the
recovered rows), then prints one JSON line per round.  Not product code.

  python3 tools/rx_frames_ab.py [rounds] [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(rounds=4, reps=12):
    import numpy as np
    import torch

    from ugo_amd import fec

    d, p, n, S, slot = 10, 3, 13, 1470, 1488
    G = 65536
    pitch_p, pitch_f, pitch_f64 = 1472, 1488, 1536  # frames64: 64-B pitch, rows written to whole lines
    dev = torch.device("cuda:0")
    enc = fec.New(d, p)
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", slot)), dtype=torch.uint8).to(dev)
    gen = torch.Generator(device=dev).manual_seed(0x5A)
    rx_id, rec_id = fec.KERNEL_IDS["rx_assemble"], fec.KERNEL_IDS["reconstruct"]

    def kernel_ms(fn, kid):
        enc.timing_begin(16 * reps)
        for r in range(reps):
            fn(r)
        recs, _ = enc.timing_end()
        return float(recs["ms"][recs["kernel"] == kid].sum()) / reps

    seq_all = torch.arange(G * n, device=dev, dtype=torch.int64)
    keep = torch.rand(G * n, device=dev, generator=gen) >= 0.05
    for order in ("in_order", "shuffled"):
        seq = seq_all[keep]
        if order == "shuffled":
            seq = seq[torch.randperm(seq.numel(), device=dev, generator=gen)]
        npk = seq.numel()
        rings = []
        for _ in range(2):
            w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
            hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
            for b in range(4):
                hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
            hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
            w[:, :6] = hdr ^ pad[:6]
            rings.append(w)
        lens = torch.full((npk,), 1476, dtype=torch.int16, device=dev)
        forms = {}
        for name, pitch, frames in (("payload", pitch_p, False), ("frames", pitch_f, True),
                                    ("frames64", pitch_f64, True)):
            forms[name] = {
                "pitch": pitch, "frames": frames,
                "bats": [torch.empty((n, G, pitch), dtype=torch.uint8, device=dev) for _ in range(2)],
                "pres": [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(2)],
                "lsts": [torch.empty(G, dtype=torch.int32, device=dev) for _ in range(2)],
                "cnts": [torch.empty(1, dtype=torch.int32, device=dev) for _ in range(2)],
                "outs": [torch.empty((G, p, pitch), dtype=torch.uint8, device=dev) for _ in range(2)],
            }

        def rx_fn(f):
            def rx(r):
                i = r % 2
                f["pres"][i].zero_()
                enc.rx_assemble(rings[i], lens, f["bats"][i], f["pres"][i], shard_size=S, pad=pad,
                                frames=f["frames"])
            return rx

        def rec_fn(f):
            W = S + 6 if f["frames"] else S

            def rec(r):
                i = r % 2
                enc.lossy_groups(f["pres"][i], data_only=True, out=f["lsts"][i], count=f["cnts"][i])
                enc.reconstruct_list(f["bats"][i], f["pres"][i], f["lsts"][i], f["cnts"][i], f["outs"][i],
                                     shard_size=W, data_only=True)
            return rec

        for f in forms.values():
            for r in range(4):
                rx_fn(f)(r)
                rec_fn(f)(r)
        torch.cuda.synchronize()
        P, F = forms["payload"], forms["frames64"]
        k = int(P["cnts"][0].item())
        ok = (torch.equal(P["pres"][0], F["pres"][0]) and k == int(F["cnts"][0].item())
              and torch.equal(P["lsts"][0][:k], F["lsts"][0][:k]))
        m = P["pres"][0]
        for r in range(n):  # payload columns of every placed row
            rows = ((m >> r) & 1).bool()
            ok = ok and torch.equal(P["bats"][0][r, rows, :S], F["bats"][0][r, rows, 6:6 + S])
            ok = ok and not bool(F["bats"][0][r, rows, S + 6:].any())
            ok = ok and torch.equal(forms["frames"]["bats"][0][r, rows, :S + 6], F["bats"][0][r, rows, :S + 6])
        pm = m[P["lsts"][0][:k].long()]
        lost = (((pm[:, None] >> torch.arange(d, device=dev)) & 1) == 0).sum(1)
        have = ((pm[:, None] >> torch.arange(n, device=dev)) & 1).sum(1)
        for i in range(p):
            sel = (lost > i) & (have >= d)
            ok = ok and torch.equal(P["outs"][0][:k][sel, i, :S], F["outs"][0][:k][sel, i, 6:6 + S])
        print(json.dumps({"order": order, "check_frames_eq_payload": bool(ok), "npk": npk, "lossy": k}), flush=True)
        rx_bytes = npk * (1476 + S)
        for rnd in range(rounds):
            line = {"order": order, "round": rnd}
            for name in (("payload", "frames", "frames64") if rnd % 2 == 0 else ("frames64", "frames", "payload")):
                f = forms[name]
                rx_ms = kernel_ms(rx_fn(f), rx_id)
                for r in range(2):
                    rx_fn(f)(r)
                rec_ms = kernel_ms(rec_fn(f), rec_id)
                line[name] = {"rx_ms": round(rx_ms, 4), "rx_frac": round(rx_bytes / (rx_ms * 1e-3) / 8e12, 4),
                              "reconstruct_list_ms": round(rec_ms, 4)}
            print(json.dumps(line), flush=True)
        del rings, forms
        torch.cuda.empty_cache()
    enc.close()


def same_storage(trials=6, reps=12):
    """Payload rows and frame rows in the SAME device storage (one flat buffer
    per cold copy, viewed at pitch 1472 or 1536), so each comparison is on one
    physical allocation; the storage is freed and re-made (after a dummy
    allocation of varying size) between trials, to sample placements."""
    import torch

    from ugo_amd import fec

    d, p, n, S, slot = 10, 3, 13, 1470, 1488
    G = 65536
    dev = torch.device("cuda:0")
    enc = fec.New(d, p)
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", slot)), dtype=torch.uint8).to(dev)
    gen = torch.Generator(device=dev).manual_seed(0x77)
    rx_id = fec.KERNEL_IDS["rx_assemble"]
    seq = torch.arange(G * n, device=dev, dtype=torch.int64)
    seq = seq[torch.rand(G * n, device=dev, generator=gen) >= 0.05]
    orders = {"in_order": seq, "shuffled": seq[torch.randperm(seq.numel(), device=dev, generator=gen)]}
    npk = seq.numel()
    lens = torch.full((npk,), 1476, dtype=torch.int16, device=dev)
    rx_bytes = npk * (1476 + S)

    def ring(sq):
        w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
        hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
        for b in range(4):
            hdr[:, b] = ((sq >> (8 * b)) & 0xFF).to(torch.uint8)
        hdr[:, 4] = torch.where(sq % n < d, 0xF1, 0xF2).to(torch.uint8)
        w[:, :6] = hdr ^ pad[:6]
        return w

    for t in range(trials):
        dummy = torch.empty((1 + 37 * t) << 20, dtype=torch.uint8, device=dev)
        flat = [torch.empty(n * G * 1536, dtype=torch.uint8, device=dev) for _ in range(2)]
        pres = [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(2)]
        line = {"trial": t, "npk": npk}
        for order, sq in orders.items():
            rings = [ring(sq) for _ in range(2)]
            res = {}
            for name in (("payload", "frames") if t % 2 == 0 else ("frames", "payload")):
                pitch, frames = (1472, False) if name == "payload" else (1536, True)
                bats = [f[:n * G * pitch].view(n, G, pitch) for f in flat]

                def rx(r, bats=bats, frames=frames):
                    i = r % 2
                    pres[i].zero_()
                    enc.rx_assemble(rings[i], lens, bats[i], pres[i], shard_size=S, pad=pad, frames=frames)

                for r in range(3):
                    rx(r)
                enc.timing_begin(16 * reps)
                for r in range(reps):
                    rx(r)
                recs, _ = enc.timing_end()
                ms = float(recs["ms"][recs["kernel"] == rx_id].sum()) / reps
                res[name] = {"ms": round(ms, 4), "frac": round(rx_bytes / (ms * 1e-3) / 8e12, 4)}
            line[order] = res
            del rings
        print(json.dumps(line), flush=True)
        del flat, pres, dummy
        torch.cuda.empty_cache()
    enc.close()


def row_pad(trials=4, reps=10):
    """Frame rows with the planar row stride padded (G*1536 + pad) on one
    allocation per trial: does a pad between the 13 row streams pick the fast
    placement mode?  Every pad is timed on the same storage in each trial."""
    import torch

    from ugo_amd import fec

    d, p, n, S, slot, G = 10, 3, 13, 1470, 1488, 65536
    pads = [0, 256, 4096, 65536 + 256, (1 << 20) + 4096, (2 << 20) + 64 * 1536]
    dev = torch.device("cuda:0")
    enc = fec.New(d, p)
    pad_ks = torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", slot)), dtype=torch.uint8).to(dev)
    gen = torch.Generator(device=dev).manual_seed(0x99)
    rx_id = fec.KERNEL_IDS["rx_assemble"]
    seq = torch.arange(G * n, device=dev, dtype=torch.int64)
    seq = seq[torch.rand(G * n, device=dev, generator=gen) >= 0.05]
    orders = {"in_order": seq, "shuffled": seq[torch.randperm(seq.numel(), device=dev, generator=gen)]}
    npk = seq.numel()
    lens = torch.full((npk,), 1476, dtype=torch.int16, device=dev)
    rx_bytes = npk * (1476 + S)
    for t in range(trials):
        dummy = torch.empty((1 + 53 * t) << 20, dtype=torch.uint8, device=dev)
        span = n * G * 1536 + (n - 1) * max(pads)
        flat = [torch.empty(span, dtype=torch.uint8, device=dev) for _ in range(2)]
        pres = [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(2)]
        line = {"trial": t}
        for order, sq in orders.items():
            rings = []
            for _ in range(2):
                w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
                hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
                for b in range(4):
                    hdr[:, b] = ((sq >> (8 * b)) & 0xFF).to(torch.uint8)
                hdr[:, 4] = torch.where(sq % n < d, 0xF1, 0xF2).to(torch.uint8)
                w[:, :6] = hdr ^ pad_ks[:6]
                rings.append(w)
            res = {}
            for pad in (pads if t % 2 == 0 else pads[::-1]):
                rs = G * 1536 + pad
                bats = [f.as_strided((n, G, 1536), (rs, 1536, 1)) for f in flat]

                def rx(r, bats=bats):
                    i = r % 2
                    pres[i].zero_()
                    enc.rx_assemble(rings[i], lens, bats[i], pres[i], shard_size=S, pad=pad_ks, frames=True)

                for r in range(3):
                    rx(r)
                enc.timing_begin(16 * reps)
                for r in range(reps):
                    rx(r)
                recs, _ = enc.timing_end()
                ms = float(recs["ms"][recs["kernel"] == rx_id].sum()) / reps
                res[str(pad)] = round(ms, 4)
            line[order] = res
            del rings
        print(json.dumps(line), flush=True)
        del flat, pres, dummy
        torch.cuda.empty_cache()
    enc.close()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "pad":
        row_pad(*(int(a) for a in sys.argv[2:4]))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "same":
        same_storage(*(int(a) for a in sys.argv[2:4]))
    else:
        main(*(int(a) for a in sys.argv[1:3]))
