#!/bin/bash
# Per-call service on the GPU box: its parity tests, the shim replay, then the
# per-group latency tool (launch path and service, same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-svc}
timeout -k 10 300 python -u -m pytest tests/test_service.py tests/test_cgo_shim_replay.py tests/test_fec_conn.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -8 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
make -C tools pergroup_latency > /dev/null 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 300 ./tools/pergroup_latency ${2:-2000} > $OUT/pergroup_$TAG.jsonl 2> $OUT/pergroup_$TAG.err
rc=$?; cat $OUT/pergroup_$TAG.jsonl | cut -c1-200; [ $rc -eq 0 ] || { echo "latency rc=$rc"; tail -5 $OUT/pergroup_$TAG.err; exit $rc; }
