#!/usr/bin/env python3
"""Per-kernel averages of every PMC counter in rocprofv3 CSV passes.

Usage: pmc_dump.py <dir> [<dir> ...]  -- each dir holds one --pmc pass
(*counter_collection.csv, any depth).  Kernels are keyed by their full
template name; counters are summed over a dispatch's rows (XCDs / SEs) and
averaged over dispatches.  Derived, when the counters are there:
  valu_per_wave      SQ_INSTS_VALU / SQ_WAVES
  valu_issue_us      SQ_INSTS_VALU x 4 cycles / 1024 SIMDs / 2.4 GHz
  valu_busy          SQ_ACTIVE_INST_VALU x 4 / (SQ_BUSY_CYCLES x SIMDs per SQ ... ) is
                     hardware-specific, so the raw counters are printed instead.
One JSON line per kernel.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS, CLOCK_HZ = 1024, 2.4e9


def short(name):
    return name.replace("void ugo::kern::", "").replace("ugo::kern::", "").split("(ugo")[0]


def main():
    per = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            disp = defaultdict(lambda: defaultdict(float))
            names = {}
            for row in csv.DictReader(open(f)):
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                names[key] = short(row["Kernel_Name"])
                disp[key][row["Counter_Name"]] += float(row["Counter_Value"])
            for key, c in disp.items():
                for n, v in c.items():
                    per[names[key]][n].append(v)
    for k in sorted(per):
        c = {n: sum(v) / len(v) for n, v in per[k].items()}
        out = {"kernel": k, "dispatches": max(len(v) for v in per[k].values())}
        out.update({n: round(v, 1) for n, v in sorted(c.items())})
        if c.get("SQ_WAVES") and "SQ_INSTS_VALU" in c:
            out["valu_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1)
            out["valu_issue_us"] = round(c["SQ_INSTS_VALU"] * 4 / SIMDS / CLOCK_HZ * 1e6, 1)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
