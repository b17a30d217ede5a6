#!/usr/bin/env python3
"""HBM traffic of the rx_tx leg's kernels over their algorithmic bytes, from a
tools/pmc_pass.sh run (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
of bench.py with the rx_tx leg).  Per kernel: the median over its dispatches
that moved data (RX's gated-off passes read nothing), hbm_read = 2 x
FETCH_SIZE x 1024 (MI355X_MICROARCH.md's gfx950 correction for wide streaming
reads), hbm_write = WRITE_SIZE x 1024.  Algorithmic bytes: RX 1476 B read +
1470 B written per packet of the leg's ring; TX 10 x 1476 read + 13 x 1476
written per group; encode / reconstruct as BASELINE.md.

  python3 tools/pmc_rxtx.py gpurun_out/pmc_<tag> <label> > profiles/<round>/pmc_rxtx.json
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

SHORT = ("k_rx_place_h", "k_rx_claim", "k_rx_begin", "k_tx_c<10", "k_encode_g", "k_apply_p<10, 1, 3",
         "k_lossy_count", "k_lossy_write", "k_packet_decode", "k_nt_copy")


def per_dispatch(d):
    per = defaultdict(float)
    name = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[key] += float(r["Counter_Value"])
            name[key] = r["Kernel_Name"]
    out = defaultdict(list)
    for key, v in per.items():
        for s in SHORT:
            if s in name[key]:
                out[s].append(v)
                break
    return out


def moved(vals):
    top = max(vals) if vals else 0.0
    return [v for v in vals if v > 0.01 * top]


def main():
    base, label = sys.argv[1], sys.argv[2]
    fetch = per_dispatch(os.path.join(base, f"{label}_FETCH_SIZE"))
    write = per_dispatch(os.path.join(base, f"{label}_WRITE_SIZE"))
    bench = {}
    p = os.path.join(base, f"{label}_FETCH_SIZE.json")
    if os.path.exists(p):
        lines = [ln for ln in open(p) if ln.strip().startswith("{")]
        bench = json.loads(lines[-1]) if lines else {}
    rt = bench.get("rx_tx", {})
    cfg = bench.get("config", {})
    npk = rt.get("rx_in_order", {}).get("packets")
    G = rt.get("tx", {}).get("groups")
    Gb, S = cfg.get("groups_per_gpu"), cfg.get("shard_size")
    alg = {}
    if npk:
        alg["k_rx_place_h"] = (npk * 1476, npk * 1470)
    if G:
        alg["k_tx_c<10"] = (G * 10 * 1476, G * 13 * 1476)
    if Gb and S:
        alg["k_encode_g"] = (Gb * 10 * S, Gb * 3 * S)
        alg["k_apply_p<10, 1, 3"] = (Gb * 10 * S, Gb * 2 * S)
    res = {}
    for k in SHORT:
        f, w = moved(fetch.get(k, [])), moved(write.get(k, []))
        if not f and not w:
            continue
        rd = 2 * statistics.median(f) * 1024 if f else 0.0
        wr = statistics.median(w) * 1024 if w else 0.0
        ent = {"dispatches_moving_data": [len(f), len(w)], "hbm_read_bytes": rd, "hbm_write_bytes": wr}
        if k in alg:
            ar, aw = alg[k]
            ent.update(alg_read_bytes=ar, alg_write_bytes=aw, read_over_alg=round(rd / ar, 4),
                       write_over_alg=round(wr / aw, 4), total_over_alg=round((rd + wr) / (ar + aw), 4))
        res[k] = ent
    res["note"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of tools/pmc_pass.sh "
                   f"(label {label}); per dispatch that moved data (median); hbm_read = 2 x FETCH_SIZE x 1024, "
                   "hbm_write = WRITE_SIZE x 1024; algorithmic: RX 1476 B read + 1470 B written per packet "
                   f"({npk} packets), TX 10 x 1476 read + 13 x 1476 written per group ({G} groups), the "
                   "encode (d+p)*S and the 2-erasure reconstruct (d+2)*S per group. The reconstruct's "
                   "median mixes the bench step's and the rx_tx leg's data-only recoveries.")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
