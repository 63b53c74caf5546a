#!/bin/bash
# face_groups (default 2): exactness incl. 3 / 4 groups; A/B over G; headline rocprof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_plates.py tests/test_gpu_e2e.py -k "face_groups or batch or micro" -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
for g in 2 3 4 1 2; do timeout -k 10 200 "${B[@]}" --option face_groups=$g > $OUT/g$g.json 2>> $OUT/bench.err || exit 1; done
for g in 3 4; do timeout -k 10 200 "${B[@]}" --plates 0 --option face_groups=$g > $OUT/faces_g$g.json 2>> $OUT/bench.err || exit 1; done
mkdir -p gpurun_out/prof_r4i
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4i -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --compare "" --host-pipeline 0 > gpurun_out/prof_r4i/bench.json 2> gpurun_out/prof_r4i/bench.err || exit 1
