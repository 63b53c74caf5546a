#!/bin/bash
# fp16 plan on the fused kernels: tests, then C3 fp16 / C5 4K fp16 lines and the default headline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 tools/x6bench 20 all > $OUT/x6.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_gpu_configs.py tests/test_gpu_plates.py tests/test_gpu_kernels.py -k "16bit or fp16 or c5 or 4k or plate" -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --precision fp16 > $OUT/c3_fp16.json 2>> $OUT/bench.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --precision fp16 --height 2160 --width 3840 --frames-src up2 > $OUT/c5_fp16.json 2>> $OUT/bench.err || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline > $OUT/bench.json 2>> $OUT/bench.err || exit 1
