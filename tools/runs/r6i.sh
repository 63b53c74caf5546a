#!/bin/bash
# pipelined block: timing-only stage skips (option block32_dbg) -> conv ms per step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6i
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 10 --warmup 2 --compare "" --no-cpu-baseline --host-pipeline 0 --plates 0 --option block32_pipe=1)
for d in 0 1 2 4 8 16 6 14 30 1 0; do
  timeout -k 10 300 "${B[@]}" --debug block32_dbg=$d > $OUT/d$d.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$OUT/d$d.json').read().strip().splitlines()[-1]);print('dbg=$d',d['ms_per_step'],d['ms_breakdown_per_step']['conv'])"
done
