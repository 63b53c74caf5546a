#!/bin/bash
# JPEG-in / JPEG-out pipeline: decode passes per host convergence check (jdec_group)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5g
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 8 --warmup 2 --compare "" --no-cpu-baseline --no-timing)
for g in 4 8 16 4; do
  timeout -k 10 300 "${B[@]}" --option jdec_group=$g > $OUT/b_$g.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json;d=json.loads(open('$OUT/b_$g.json').read().strip().splitlines()[-1]);j=d['jpeg_pipeline'];s=d['jpeg_pipeline_structured'];print('jdec_group=$g',d['ms_per_step'],'noise',j['value'],j['stage_ms_per_step'],j['decode_sync_passes'],'structured',s['value'],s['stage_ms_per_step'])"
done
