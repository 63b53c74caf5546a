#!/bin/bash
# x6_one: bit-identity test, x6bench layer A/B, headline A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "x6_one or fused_layer1" -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
X6_TAG=r4w_x6 X6_RUNS="one:;tap:x6_one=0;one2:;tap2:x6_one=0" bash tools/runs/x6.sh > $OUT/x6.txt 2>&1 || { tail -5 $OUT/x6.txt; exit 1; }
grep -E "==|total" $OUT/x6.txt
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
run() { local tag=$1; shift; timeout -k 10 200 "${B[@]}" "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.json)"; }
for r in 1 2; do
  run one_$r
  run tap_$r --option x6_one=0
done
