#!/bin/bash
# GpuJpegStages serial-decode test + JPEG pipeline lines (auto schedule)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B=(python bench.py --steps 8 --warmup 2 --compare "" --no-cpu-baseline --no-timing)
for r in 1 2; do
  timeout -k 10 300 "${B[@]}" > $OUT/b_$r.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json;d=json.loads(open('$OUT/b_$r.json').read().strip().splitlines()[-1]);j=d['jpeg_pipeline'];s=d['jpeg_pipeline_structured'];print('run $r',d['ms_per_step'],'noise',j['value'],j['stage_ms_per_step'],j['serial_decode_jobs'],'structured',s['value'],s['stage_ms_per_step'],s['serial_decode_jobs'])"
done
