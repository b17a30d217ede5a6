#!/bin/bash
# TX traffic attribution on the GPU box: tools/txpmc timed,
# then one rocprofv3 PMC pass per counter group, for 16-B slots (1488) and
# 128-B aligned slots (1536); per-kernel averages into gpurun_out/txpmc/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/txpmc
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
EXTRA=""
if grep -q "TCC_EA0_RDREQ_32B" "$OUT/avail.txt" && grep -q "TCC_EA0_RDREQ\b\|TCC_EA0_RDREQ[^_]" "$OUT/avail.txt"; then
  EXTRA="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum"
fi
for slot in 1488 1536; do
  timeout -k 10 90 tools/txpmc 15 $slot > "$OUT/time_$slot.jsonl" 2> "$OUT/time_$slot.err" || { echo "txpmc $slot failed"; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE "$EXTRA"; do
    [ -n "$ctr" ] || continue
    tag=$(echo $ctr | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/${slot}_$tag" -o run -- tools/txpmc 15 $slot \
      > "$OUT/${slot}_$tag.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $slot $tag rc=$rc"; tail -3 "$OUT/${slot}_$tag.log"; exit $rc; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
res = {}
for d in sorted(glob.glob(out + "/*_*/")):
    slot, tag = os.path.basename(d.rstrip("/")).split("_", 1)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            name[key] = r["Kernel_Name"]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for key, cs in per.items():
        for c, v in cs.items():
            agg[name[key]][c].append(v)
    for k, cs in agg.items():
        import re
        mm = re.search(r"(k_\w+)(<[^(]*>)?", k)
        short = (mm.group(1) + (mm.group(2) or "")) if mm else k[:60]
        for c, v in cs.items():
            v = sorted(v)
            res.setdefault(slot, {}).setdefault(short, {})[c] = v[len(v) // 2]
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
