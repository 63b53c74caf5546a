#!/bin/bash
# pipelined layer1 block iteration: fp32 block parity, bench A/B, rocprof layer view
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${R6F_TAG:-r6f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_e2e.py -k "bottleneck_fp32 or block32_pipe" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { tail -30 $OUT/tests.log; exit $rc; }
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
show() { python3 -c "
import json;d=json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1]);print('$1',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['per_launch']['frac'])"; }
for pp in 1 0; do
  timeout -k 10 300 "${B[@]}" --option block32_pipe=$pp > $OUT/p${pp}.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  show p${pp}
done
PROF_TAG=${R6F_TAG:-r6f}/prof timeout -k 10 600 tools/runs/prof.sh > /dev/null
grep -E "l1\.|total" gpurun_out/${R6F_TAG:-r6f}/prof/layers.txt
