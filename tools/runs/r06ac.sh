#!/bin/bash
# headline repeat on one box, final code: five back-to-back bench lines (value, ms/step, frac, per-launch frac, blur frac)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06ac
export TMPDIR=/tmp
for r in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 > gpurun_out/r06ac/b$r.json 2>> gpurun_out/r06ac/err.log || { tail -20 gpurun_out/r06ac/err.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06ac/b$r.json').read().strip().splitlines()[-1]);print('run $r',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['per_launch']['frac'],d['blur_roofline']['frac'])"
done
