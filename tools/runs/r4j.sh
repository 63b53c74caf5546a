#!/bin/bash
# face_groups = 2: lag sweep (face_group_lag) and plate release point sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4j
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
for l in 0 1 4 10 17 0; do timeout -k 10 200 "${B[@]}" --option face_group_lag=$l > $OUT/lag$l.json 2>> $OUT/bench.err || exit 1; echo "lag $l $(tail -c 300 $OUT/lag$l.json | grep -o '"ms_per_step": [0-9.]*')"; done
for p in 0 1 2 4 5; do timeout -k 10 200 "${B[@]}" --option plate_stage=$p > $OUT/ps$p.json 2>> $OUT/bench.err || exit 1; echo "ps $p $(grep -o '"ms_per_step": [0-9.]*' $OUT/ps$p.json)"; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_plates.py -k "face_groups" -p no:cacheprovider > $OUT/tests.log 2>&1; tail -2 $OUT/tests.log
