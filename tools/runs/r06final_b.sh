#!/bin/bash
# round-6 final set, part B: rocprof of the headline (with its instrumented pass) + per-layer view, PMC traffic
# (face_groups=1), SQ counters, step timeline, faces-only / C2 bf16 / C5 4K fp16 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06final
mkdir -p $OUT
T=r06final/prof
mkdir -p gpurun_out/$T
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
S=$(find gpurun_out/$T -name 'run_kernel_stats.csv' | head -1)
K=$(find gpurun_out/$T -name 'run_kernel_trace.csv' | head -1)
tail -1 gpurun_out/$T/bench.json > gpurun_out/$T/line.json
python tools/prof_summary.py "$S" gpurun_out/$T/summary.md gpurun_out/$T/line.json > /dev/null 2>&1 || true
python tools/fp32_layers.py "$K" 64 1 > gpurun_out/$T/layers.txt 2>&1 || true
python tools/step_timeline.py $(dirname "$K") > gpurun_out/$T/timeline.txt 2>&1 || true
tail -4 gpurun_out/$T/summary.md
PMC_TAG=r06final/pmc BARGS="--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --option face_groups=1" timeout -k 10 500 tools/runs/pmc.sh || exit 1
SQ_TAG=r06final/sq BARGS="--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --option face_groups=1 --plates 0" timeout -k 10 500 tools/runs/sq.sh > $OUT/sq.txt 2>&1 || { tail -5 $OUT/sq.txt; exit 1; }
timeout -k 10 300 python bench.py --plates 0 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/faces.json 2>> $OUT/err.log || exit 1
timeout -k 10 300 python bench.py --height 720 --width 1280 --batch 32 --precision bf16 --frames-src up2 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/c2_bf16.json 2>> $OUT/err.log || exit 1
timeout -k 10 300 python bench.py --height 2160 --width 3840 --batch 64 --precision fp16 --frames-src up2 --steps 10 --warmup 2 --compare "" --no-cpu-baseline --host-pipeline 0 > $OUT/c5_fp16.json 2>> $OUT/err.log || exit 1
for f in faces c2_bf16 c5_fp16; do python3 -c "
import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],d['blur_roofline']['frac'])"; done
