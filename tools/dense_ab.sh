#!/bin/bash
# Dense planar rows (pitch == S) against the padded 16-B pitch: parity tests of
# the dense paths, then the bench step at both pitches, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-dense}
REPS=${2:-2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "dense or shard_major or reconstruct_into_vs or encode_10_3" > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -5 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
bash tools/bench_ab.sh $TAG $REPS "pad|--pitch 1360" "dense|--pitch 1350"
