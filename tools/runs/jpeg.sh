#!/bin/bash
# JPEG legs: GPU codec tests, then the bench's jpeg_pipeline figure (headline run trimmed)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${JPEG_TAG:-jpeg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_jpeg.py -p no:cacheprovider ${PYTEST_EXTRA:-} > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --compare '' --no-cpu-baseline --no-timing ${BARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['jpeg_pipeline'])"
