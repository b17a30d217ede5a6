#!/bin/bash
# GPU tests, then bench with in-place vs out-of-place (reconstruct_into) decode,
# interleaved, 2 passes.  Each GPU step has its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/decode_ab.jsonl; : > $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_into.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu_into.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_into.log
for pass in 1 2; do
  for mode in inplace into; do
    timeout -k 10 120 python bench.py --decode $mode --no-cpu-baseline > gpurun_out/dab.json 2> gpurun_out/dab.err \
      || { echo "bench $mode rc=$?"; tail -5 gpurun_out/dab.err; exit 1; }
    python -c "
import json; r=json.load(open('gpurun_out/dab.json')); k=r['kernels']
print(json.dumps({'decode': '$mode', 'pass': $pass, 'value': r['value'], 'ms_per_step': r['ms_per_step'],
 'enc_us': round(k['encode']['avg_ms']*1e3,1), 'dec_us': round(k['reconstruct']['avg_ms']*1e3,1),
 'dec_frac': k['reconstruct']['frac'], 'verify': r['verify']}))" >> $OUT
    tail -1 $OUT
  done
done
