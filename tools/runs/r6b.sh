#!/bin/bash
# product-path sharding: new shard tests, pipeline + bench-dist tests, then a quick headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_shard.py tests/test_gpu_pipeline.py tests/test_gpu_bench_dist.py tests/test_gpu_dist.py > $OUT/tests.log 2>&1; rc=$?
tail -30 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/head.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/head.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['step'])"
