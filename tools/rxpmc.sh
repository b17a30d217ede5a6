#!/bin/bash
# RX instruction / request mix (round 5): rocprofv3 PMC passes over tools/rxgather
# (production placement and the compute-free access patterns of the same ring),
# one pass per counter group, per-kernel-and-grid averages into gpurun_out/rxpmc/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export RXG_ONLY="gated claim / re-place on 1024"
OUT=$PWD/gpurun_out/rxpmc
mkdir -p "$OUT"
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
            "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_ANY"; do
  i=$((i+1))
  for ord in inorder shuffled; do
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/p${i}_$ord" -o run -- tools/rxgather 3 $ord \
      > "$OUT/p${i}_$ord.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pass $i $ord rc=$rc"; tail -3 "$OUT/p${i}_$ord.log"; exit $rc; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(dict))
for d in sorted(glob.glob(out + "/p*_*/")):
    ordr = os.path.basename(d.rstrip("/")).split("_", 1)[1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    key_of = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[disp][r["Counter_Name"]] += float(r["Counter_Value"])
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ugo::kern::", "")
            key_of[disp] = f"{name} grid={r.get('Grid_Size', '?')}"
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for disp, cs in per.items():
        for c, v in cs.items():
            agg[key_of[disp]][c].append(v)
    for k, cs in agg.items():
        for c, v in cs.items():
            res[ordr][k][c] = sum(v) / len(v)
            res[ordr][k]["dispatches"] = len(v)
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print("ok")
PY
