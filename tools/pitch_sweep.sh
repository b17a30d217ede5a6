#!/bin/bash
# Row-pitch sweep of the bench step (cold regime, 2 batches): does a
# 64/128-B aligned pitch cut the partial-line writes of the reconstruct?
# Interleaved: every pitch once per pass, 2 passes.  Each run has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pitch_sweep.jsonl
mkdir -p gpurun_out; : > $OUT
for pass in 1 2; do
  for pitch in ${PITCHES:-1360 1408 1472 1536}; do
    timeout -k 10 120 python bench.py --pitch $pitch --no-cpu-baseline --steps 200 --warmup 50 \
      > gpurun_out/ps.json 2> gpurun_out/ps.err || { echo "pitch $pitch rc=$?"; tail -5 gpurun_out/ps.err; exit 1; }
    python - "$pitch" "$pass" >> $OUT <<'PY'
import json, sys
r = json.load(open("gpurun_out/ps.json"))
k = r["kernels"]
print(json.dumps({"pitch": int(sys.argv[1]), "pass": int(sys.argv[2]), "value": r["value"],
                  "ms_per_step": r["ms_per_step"], "enc_us": round(k["encode"]["avg_ms"] * 1e3, 1),
                  "dec_us": round(k["reconstruct"]["avg_ms"] * 1e3, 1), "verify": r["verify"]}))
PY
    tail -1 $OUT
  done
done
