#!/bin/bash
# pipelined block: stage-1 x depth (block32_pipe = 1 (3 sets) / 4 / 5 / 6) vs the one-group kernel (0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "bottleneck_fp32" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
B=(python bench.py --steps 10 --warmup 2 --compare "" --no-cpu-baseline --host-pipeline 0 --plates 0)
for r in 1 2; do
for pp in 0 1 4 5 6; do
  timeout -k 10 300 "${B[@]}" --option block32_pipe=$pp > $OUT/p$pp.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$OUT/p$pp.json').read().strip().splitlines()[-1]);print('pipe=$pp',d['ms_per_step'],d['ms_breakdown_per_step']['conv'])"
done
done
