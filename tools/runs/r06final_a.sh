#!/bin/bash
# round-6 final set, part A: full GPU suite + smoke, then the default bench line (as the driver runs it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SUITE_TAG=r06final/suite bash tools/runs/suite.sh || exit 1
OUT=gpurun_out/r06final
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['per_launch']['frac'],d['blur_roofline']['frac'],d['jpeg_pipeline']['value'],d['jpeg_pipeline_structured']['value'],d['cpu_baseline']['value'],d.get('parity'))"
