#!/bin/bash
# rocprofv3 evidence for the jumbo (32+8)x9000 calls of tools/bench_host.py:
#   1. --kernel-trace --stats      -> per-kernel durations
#   2. --pmc SQ_* GRBM_GUI_ACTIVE  -> VALU instructions per wave (own pass)
# PMC never combines with trace domains.  Summary: tools/pmc_kernels.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-jumbo}
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/bench_host.py --only jumbo --reps 5 > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/sq" -o run -- python3 tools/bench_host.py --only jumbo --reps 5 \
  > "$OUT/sq.log" 2>&1 || { echo "sq rc=$?"; exit 1; }
python3 tools/pmc_kernels.py "$OUT" > "$OUT/summary.jsonl"
cat "$OUT/summary.jsonl"
