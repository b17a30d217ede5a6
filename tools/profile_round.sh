#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box via gpurun):
#   1. --kernel-trace --stats          -> per-kernel average duration
#   2. --pmc FETCH_SIZE                -> HBM read bytes   (own pass)
#   3. --pmc WRITE_SIZE                -> HBM write bytes  (own pass)
#   4. --pmc SQ_* (VALU / wave cycles) -> issue utilisation (own pass)
# PMC passes never combine with sys/runtime/hip/hsa trace domains.
# Then tools/pmc_traffic.py summarises everything into profiles/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r1}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 40 --warmup 50 --no-verify --no-cpu-baseline --no-host-path --no-rx-tx --c4-total-groups 0 ${BENCH_EXTRA:-}"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 bench.py $ARGS \
    > "$OUT/$name.bench.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"; tail -2 "$OUT/$name.err"
  return $rc
}
run trace --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || echo "sq pass failed (non-fatal)"
python3 tools/pmc_traffic.py "$OUT" "$TAG"
