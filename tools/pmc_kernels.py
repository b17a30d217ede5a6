#!/usr/bin/env python3
"""Per-kernel VALU roof from a tools/pmc_jumbo.sh run (any rocprofv3 CSV pair).

Inputs (<dir>/trace: --kernel-trace --stats; <dir>/sq: --pmc SQ_WAVES
SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE).  For every
kernel name: dispatches, average duration, VALU instructions per wave, and the
VALU issue time = VALU/wave x waves x 4 cycles / 1024 SIMDs / 2.4 GHz (a wave64
VALU instruction occupies a SIMD for 4 cycles), the "both roofs" table of
DESIGN_HISTORY.md §4.  One JSON line per kernel on stdout.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS, CLOCK_HZ = 1024, 2.4e9


def short(name):
    base = name.split("(")[0]
    return base.replace("void ugo::kern::", "").replace("ugo::kern::", "")


def main():
    d = sys.argv[1]
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            dur[short(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    cnt = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for f in glob.glob(os.path.join(d, "sq", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            key = (short(row["Kernel_Name"]), row.get("Dispatch_Id") or row.get("Correlation_Id"))
            cnt[key][row["Counter_Name"]] += float(row["Counter_Value"])
    per = defaultdict(lambda: defaultdict(list))
    for (k, _), c in cnt.items():
        for n, v in c.items():
            per[k][n].append(v)
    for k in sorted(set(dur) | set(per)):
        c = {n: sum(v) / len(v) for n, v in per[k].items()}
        waves = c.get("SQ_WAVES", 0.0)
        valu = c.get("SQ_INSTS_VALU", 0.0)
        out = {"kernel": k, "dispatches": len(dur.get(k, [])),
               "avg_us": round(sum(dur[k]) / len(dur[k]), 2) if dur.get(k) else None}
        if waves:
            out["valu_per_wave"] = round(valu / waves, 1)
            out["valu_issue_us"] = round(valu * 4 / SIMDS / CLOCK_HZ * 1e6, 1)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
