#!/bin/bash
# paired letterbox in every plan; headline with block32 / mosaic defaults restored; faces-only
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_plates.py tests/test_gpu_kernels.py -k "paired or block32 or layer1" -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/bench$i.json 2>> $OUT/bench.err || exit 1; done
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --plates 0 > $OUT/faces.json 2>> $OUT/bench.err || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --option lb_pair=0 > $OUT/nopair.json 2>> $OUT/bench.err || exit 1
