#!/bin/bash
# pipelined layer1 block: parity tests, bench A/B, rocprof layer view
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_e2e.py -k "bottleneck or layer1 or block32 or ssh" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|fp32 bottleneck" $OUT/tests.log | tail -20
[ $rc -eq 0 ] || { tail -30 $OUT/tests.log; exit $rc; }
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
show() { python3 -c "
import json;d=json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1]);print('$1',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['per_launch']['frac'],d['ms_breakdown_per_step'])"; }
for r in 1 2; do
  for pp in 1 0; do
    timeout -k 10 300 "${B[@]}" --option block32_pipe=$pp > $OUT/p${pp}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    show p${pp}_$r
  done
done
PROF_TAG=r6e/prof timeout -k 10 600 tools/runs/prof.sh
grep -E "l1\.|total" gpurun_out/r6e/prof/layers.txt
