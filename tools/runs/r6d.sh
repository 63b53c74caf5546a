#!/bin/bash
# JPEG pipeline vs hardware queues; C2 bf16 and C5 4K fp16 lines (fused mosaic)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6d
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline)
show() { python3 -c "
import json;d=json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1]);j=d.get('jpeg_pipeline',{});s=d.get('jpeg_pipeline_structured',{})
print('$1',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline'].get('per_launch',{}).get('frac'),d['blur_roofline']['frac'],j.get('value'),j.get('stage_ms_per_step'),s.get('value'))"; }
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 "${B[@]}" > $OUT/q$q.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  show q$q
done
timeout -k 10 300 python bench.py --height 720 --width 1280 --batch 32 --precision bf16 --frames-src up2 --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/c2.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
show c2
timeout -k 10 300 python bench.py --height 2160 --width 3840 --batch 64 --precision fp16 --frames-src up2 --steps 10 --warmup 2 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/c5.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
show c5
