#!/bin/bash
# round-5 measurement set: default bench line, rocprof stats + per-layer view, PMC traffic
# (fp32 headline), faces-only line, C2 bf16 and C5 4K fp16 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['per_launch'],d['blur_roofline']['frac'],d['jpeg_pipeline']['value'],d['jpeg_pipeline_structured']['value'],d['cpu_baseline']['value'],d.get('parity'))"
PROF_TAG=r6final/prof timeout -k 10 600 tools/runs/prof.sh || exit 1
PMC_TAG=r6final/pmc timeout -k 10 700 tools/runs/pmc.sh || exit 1
timeout -k 10 300 python bench.py --plates 0 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/faces.json 2>> $OUT/err.log || exit 1
timeout -k 10 300 python bench.py --height 720 --width 1280 --batch 32 --precision bf16 --frames-src up2 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/c2_bf16.json 2>> $OUT/err.log || exit 1
timeout -k 10 300 python bench.py --height 2160 --width 3840 --batch 64 --precision fp16 --frames-src up2 --steps 10 --warmup 2 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/c5_fp16.json 2>> $OUT/err.log || exit 1
for f in faces c2_bf16 c5_fp16; do python3 -c "
import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],d['blur_roofline']['frac'])"; done
