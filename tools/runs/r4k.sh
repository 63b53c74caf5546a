#!/bin/bash
# fp32 plate TAPS streaming form: parity tests, plate-only A/B, headline A/B, plate rocprof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_plates.py -k "taps or raw_fp32 or post_exact or paired" -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
for t in 1 0; do timeout -k 10 200 "${B[@]}" --faces 0 --plates 1 --option x6_taps=$t > $OUT/plates_t$t.json 2>> $OUT/bench.err || exit 1; echo "plates taps=$t $(grep -o '"ms_per_step": [0-9.]*' $OUT/plates_t$t.json)"; done
for t in 1 0 1; do timeout -k 10 200 "${B[@]}" --option x6_taps=$t > $OUT/head_t$t.json 2>> $OUT/bench.err || exit 1; echo "head taps=$t $(grep -o '"ms_per_step": [0-9.]*' $OUT/head_t$t.json)"; done
mkdir -p gpurun_out/profp_r4k
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profp_r4k -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 --faces 0 --plates 1 --no-timing > gpurun_out/profp_r4k/bench.log 2>&1 || exit 1
