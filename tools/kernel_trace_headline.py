"""Average duration of the headline-size (10,3) encode / reconstruct launches in a rocprofv3
--kernel-trace of bench.py (launches of 150-260 us: the 65,536-group batch; the other legs' launches
are smaller or larger).  Not product code.

  python3 tools/kernel_trace_headline.py <rocprofv3 output dir>
"""
import csv, glob, json, sys, statistics
d = sys.argv[1]
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
out = {}
for key in ("k_encode_g<10, 3", "k_apply_p<10, 1, 3"):
    ds = [t for n, t in rows if key in n]
    big = [t for t in ds if 150 < t < 260]  # the headline batch's launches (65,536 groups)
    out[key] = {"launches": len(ds), "headline_launches": len(big),
                "headline_avg_us": round(statistics.mean(big), 2) if big else None,
                "headline_median_us": round(statistics.median(big), 2) if big else None}
print(json.dumps(out))
