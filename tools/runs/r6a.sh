#!/bin/bash
# round-5 baseline: headline bench at HEAD (no cpu baseline) + faces-only line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6a
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline)
timeout -k 10 400 "${B[@]}" > $OUT/head.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/head.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['step'],d['blur_roofline']['frac'],d['blur_roofline']['family'],d['ms_breakdown_per_step'],d['jpeg_pipeline']['value'],d['jpeg_pipeline']['stage_ms_per_step'],d['jpeg_pipeline_structured']['value'])"
