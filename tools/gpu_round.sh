#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench (rocprofv3 evidence: tools/profile_round.sh).
# Every GPU step has its own time limit; the chain stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r1}
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
rc=$?; cat $OUT/smoke_$TAG.log | tail -5; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== bench"; timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
exit 0
