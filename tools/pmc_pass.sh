#!/bin/bash
# One traffic comparison on the GPU box: FETCH_SIZE / WRITE_SIZE passes of the
# bench for each "label|bench args" given, per-kernel averages printed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
for v in "$@"; do
  label=${v%%|*}; args=${v#*|}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/${label}_$ctr" -o run -- python3 bench.py \
      --steps 20 --warmup 20 --no-verify --no-cpu-baseline --no-host-path --c4-total-groups 0 $args \
      > "$OUT/${label}_$ctr.json" 2> "$OUT/${label}_$ctr.err"
    rc=$?; [ $rc -eq 0 ] || { echo "$label $ctr rc=$rc"; tail -3 "$OUT/${label}_$ctr.err"; exit $rc; }
    python3 - "$OUT/${label}_$ctr" "$label" "$ctr" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float)
name = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[key] += float(r["Counter_Value"])  # sum over XCC / SE instances
        name[key] = r["Kernel_Name"][:60]
agg = collections.defaultdict(list)
for key in sorted(per, key=int):
    agg[name[key]].append(per[key])
for k, v in sorted(agg.items()):
    if len(v) >= 10:
        print(sys.argv[2], sys.argv[3], k, len(v), round(sum(v[-20:]) / len(v[-20:]) * 1024 / 1e6, 2), "MB(raw KiB x 1024)")
PY
  done
done
