#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/<tag>/.

Inputs (gpurun_out/prof_<tag>/): rocprofv3 CSV output of
  trace/  --kernel-trace --stats   (kernel_stats.csv)
  fetch/  --pmc FETCH_SIZE         (counter_collection.csv)
  write/  --pmc WRITE_SIZE
  sq/     --pmc SQ_* GRBM_GUI_ACTIVE
HBM traffic per launch follows MI355X_MICROARCH.md (HBM section):
  FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports exactly half
  the bytes of a wide (16 B/lane) coalesced streaming read, so
  hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Outputs: profiles/<tag>/kernel_stats.csv (copied), profiles/<tag>/pmc_summary.json,
and profiles/pmc_traffic.json (per-launch corrected traffic, read by bench.py).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KERNELS = {"k_encode_c": "encode", "k_encode_g": "encode", "k_encode_frs": "encode", "k_apply_p<": "reconstruct", "k_apply_pd<": "reconstruct", "k_apply_w<": "reconstruct", "k_apply<": "reconstruct", "k_apply_bytes": "reconstruct_bytes",
           "k_prepare": "prepare",
           # the rx_tx leg and the ceilings (round 4)
           "k_rx_place": "rx_place", "k_rx_chunk": "rx_chunk", "k_rx_begin": "rx_begin", "k_rx_count": "rx_count",
           "k_rx_claim": "rx_claim", "k_tx_g": "tx", "k_tx_c": "tx", "k_packet_decode": "packet_decode",
           "k_encode_twin": "encode_twin", "k_reconstruct_twin": "reconstruct_twin", "k_nt_copy": "nt_copy"}
BENCH_KINDS = ("encode", "reconstruct")  # the kinds whose last `steps` dispatches are the bench's timed steps


def kind(name):
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


def counters(d):
    vals = defaultdict(lambda: defaultdict(list))  # kind -> counter -> [per-dispatch values]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for row in csv.DictReader(open(f)):
            k = kind(row.get("Kernel_Name", ""))
            if not k:
                continue
            key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), row["Counter_Name"])
            per[key] += float(row["Counter_Value"])  # sum over dimensions (XCC / SE instances)
            names[key] = k
        for (disp, cname), v in per.items():
            vals[names[(disp, cname)]][cname].append(v)
    return vals


def main():
    src, tag = sys.argv[1], sys.argv[2]
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, "kernel_stats.csv"))
    # per-dispatch durations: the bench's timed steps are the LAST `steps`
    # dispatches of each kernel (the warmup dispatches before them run while
    # the clocks ramp), so report that average beside rocprof's all-dispatch one
    timed = {}
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True):
        durs = defaultdict(list)
        for row in csv.DictReader(open(f)):
            k = kind(row["Kernel_Name"])
            if k:
                durs[(k, row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        for (k, name), v in durs.items():
            timed[k] = {"kernel": name, "dispatches": len(v), "all_avg_ns": sum(v) / len(v)}
    bench = {}
    for f in glob.glob(os.path.join(src, "trace.bench.json")):
        lines = [ln for ln in open(f) if ln.strip().startswith("{")]
        if lines:
            bench = json.loads(lines[-1])
    cfg = bench.get("config", {})
    G, d, p, S, e = (cfg.get(k) for k in ("groups_per_gpu", "data_shards", "parity_shards", "shard_size", "erasures"))
    pitch = cfg.get("pitch")
    alg = {"encode": G * (d + p) * S, "reconstruct": G * (d + e) * S} if G else {}
    steps = bench.get("steps")
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True):
        durs = defaultdict(list)
        for row in csv.DictReader(open(f)):
            k = kind(row["Kernel_Name"])
            if k:
                durs[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        for k, v in durs.items():
            if k in BENCH_KINDS and steps and len(v) >= steps:
                timed[k]["timed_steps"] = steps
                timed[k]["timed_avg_ns"] = sum(v[-steps:]) / steps
    summary = {"tag": tag, "bench_config": cfg, "kernels": {}, "dispatch_durations": timed}
    merged = defaultdict(dict)
    for sub in ("fetch", "write", "sq"):
        for k, cs in counters(os.path.join(src, sub)).items():
            for cname, v in cs.items():
                merged[k][cname] = sum(v) / len(v)
                merged[k][cname + "_dispatches"] = len(v)
    traffic = {}
    for k, cs in merged.items():
        ent = dict(cs)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            raw = (cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            corr = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            ent["hbm_bytes_raw"] = raw
            ent["hbm_bytes_corrected"] = corr
            if k in alg:
                ent["algorithmic_bytes"] = alg[k]
                ent["traffic_over_algorithmic"] = corr / alg[k]
                into = ":into" if (k == "reconstruct" and cfg.get("decode") == "into") else ""
                traffic[f"{k}:{d}+{p}x{S}/{pitch}:G{G}{into}"] = corr
        summary["kernels"][k] = ent
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    old = json.load(open(tp)) if os.path.exists(tp) else {}
    old.update(traffic)
    json.dump(old, open(tp, "w"), indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
