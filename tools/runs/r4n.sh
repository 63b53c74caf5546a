#!/bin/bash
# chain32 A/B: off / layer2 only / layer2 + 3, headline and faces only
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
for r in 1 2; do for c in 0 2 1; do timeout -k 10 200 "${B[@]}" --option chain=$c > $OUT/c${c}_$r.json 2>> $OUT/bench.err || exit 1; echo "chain=$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/c${c}_$r.json)"; done; done
for c in 0 2 1; do timeout -k 10 200 "${B[@]}" --plates 0 --option chain=$c > $OUT/f${c}.json 2>> $OUT/bench.err || exit 1; echo "faces chain=$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/f${c}.json)"; done
