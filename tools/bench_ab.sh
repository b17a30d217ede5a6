#!/bin/bash
# Interleaved bench.py A/B on one box: bench_ab.sh TAG REPS "label|args" ...
# Each variant runs the main line only (no CPU baseline, host path or strong
# leg); one summary line per run: label value ms/step encode(us,frac) reconstruct(us,frac) verify.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=$1; REPS=$2; shift 2
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    label=${v%%|*}; args=${v#*|}
    envs=""; rest=""
    for t in $args; do  # leading VAR=value tokens are environment for the run
      if [ -z "$rest" ] && [[ "$t" == *=* && "$t" != -* ]]; then envs="$envs $t"; else rest="$rest $t"; fi
    done
    f=$OUT/ab_${TAG}_${label}_$rep
    timeout -k 10 180 env $envs python bench.py $rest --no-cpu-baseline --no-host-path --c4-total-groups 0 > $f.json 2> $f.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $label rc=$rc"; tail -5 $f.err; exit $rc; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], round(k['encode']['avg_ms']*1e3,1), k['encode']['frac'], round(k['reconstruct']['avg_ms']*1e3,1), k['reconstruct']['frac'], all(d['verify'].values()))" $f.json $label
  done
done
