"""Per-kernel split of reconstruct_into for codes past the host table (d+p >
16): k_prepare (kernel id 3) against the apply kernel (id 2), from the
library's launch timing, 10 calls after 20 untimed.  One JSON line per code
(profiles/r2/prep_share.jsonl)."""
import sys, os, json, torch
sys.path.insert(0, os.getcwd())
from ugo_amd import fec
for d, p, S in [(16, 4, 1350), (20, 5, 1350), (24, 8, 1350), (12, 4, 1350), (32, 8, 9000)]:
    n = d + p; pitch = (S + 15) // 16 * 16
    G = max(256, int(1.2e9 / (n * pitch)))
    enc = fec.New(d, p)
    b = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device="cuda")
    out = torch.empty((p, G, pitch), dtype=torch.uint8, device="cuda")
    gen = torch.Generator().manual_seed(1)
    m = torch.full((G,), (1 << n) - 1, dtype=torch.int64)
    e = torch.randint(1, p + 1, (G,), generator=gen)
    for g in range(G):
        for r in torch.randperm(n, generator=gen)[: int(e[g])].tolist():
            m[g] &= ~(1 << r)
    m = m.cuda()
    for _ in range(20):
        enc.reconstruct_into(b, m, out, S, shard_major=True)
    torch.cuda.synchronize()
    enc.timing_begin(64)
    for _ in range(10):
        enc.reconstruct_into(b, m, out, S, shard_major=True)
    recs, _ = enc.timing_end()
    ks = {}
    for k, ms in zip(recs["kernel"], recs["ms"]):
        ks.setdefault(int(k), []).append(float(ms))
    print(json.dumps({"d": d, "p": p, "G": G, **{str(k): round(sum(v) / len(v) * 1e3, 1) for k, v in ks.items()}}), flush=True)
