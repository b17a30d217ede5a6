#!/bin/bash
# RX placement, payload rows (k_rx_place_h) vs frame rows (k_rx_frame_h), on the same
# storage (tools/rx_frames_ab.py same): rocprofv3 PMC passes, one per counter group,
# per-kernel averages per packet into gpurun_out/rxpmc_frames/summary.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/rxpmc_frames
mkdir -p "$OUT"
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
            "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/p$i" -o run -- python3 tools/rx_frames_ab.py same 1 6 \
    > "$OUT/p$i.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -3 "$OUT/p$i.log"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
npk = json.loads([l for l in open(out + "/p1.log") if l.startswith("{")][-1])["npk"]
res = collections.defaultdict(dict)
for d in sorted(glob.glob(out + "/p*/")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    key_of, grid = {}, {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[disp][r["Counter_Name"]] += float(r["Counter_Value"])
            key_of[disp] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ugo::kern::", "")
            grid[disp] = int(r.get("Grid_Size") or 0)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for disp, cs in per.items():
        # the placement launches only (the gated re-place launch of the same kernel, on 1024 blocks, idles)
        if ("k_rx_place_h" in key_of[disp] or "k_rx_frame_h" in key_of[disp]) and grid[disp] > 1024 * 256:
            for c, v in cs.items():
                agg[key_of[disp]][c].append(v)
    for k, cs in agg.items():
        for c, v in cs.items():
            # two orders per run (in order, shuffled): the average over both, per packet
            res[k][c + "_per_packet"] = round(sum(v) / len(v) / npk, 3)
            res[k]["dispatches"] = len(v)
for k in res:
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        if c + "_per_packet" in res[k]:
            res[k][c + "_bytes_per_packet"] = round(res[k].pop(c + "_per_packet") * 1024 * (2 if c == "FETCH_SIZE" else 1), 1)
json.dump({"npk": npk, "note": "per packet, averaged over the in-order and shuffled rings of one allocation; FETCH x2 "
           "(gfx950 correction, MI355X_MICROARCH.md), x1024 (KiB units)", "kernels": res},
          open(out + "/summary.json", "w"), indent=1)
print("ok")
PY
