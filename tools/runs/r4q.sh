#!/bin/bash
# SSH conv5X5_2 + conv7X7_2 fused (ssh_fuse=2) + padded-K 1x1 on TAPS: parity tests, A/B, layer view
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_plates.py -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
for f in 1 0; do timeout -k 10 200 "${B[@]}" --faces 0 --plates 1 --option det_group=$f > $OUT/dg$f.json 2>> $OUT/bench.err || exit 1; echo "plates det_group=$f $(grep -o '"ms_per_step": [0-9.]*' $OUT/dg$f.json)"; done
for t in 1 0; do timeout -k 10 200 "${B[@]}" --faces 0 --plates 1 --option x6_taps=$t > $OUT/p$t.json 2>> $OUT/bench.err || exit 1; echo "plates taps=$t $(grep -o '"ms_per_step": [0-9.]*' $OUT/p$t.json)"; done
PROF_TAG=prof_r4q BARGS="--steps 5 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0" bash tools/runs/prof.sh > /dev/null || exit 1
