#!/bin/bash
# round-4 measurement set: default bench line, headline rocprof (timed steps in face
# groups + the face_groups=1 instrumented pass), PMC traffic and SQ counters of the
# face_groups=1 launches, C5 (4K fp16) line + rocprof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${R4L_TAG:-r4l}
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
tail -c 400 $O/bench_default.json
PROF_TAG=prof_${R4L_TAG:-r4l} BARGS="--steps 10 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0" bash tools/runs/prof.sh || exit 1
python tools/prof_summary.py gpurun_out/prof_${R4L_TAG:-r4l}/run_kernel_stats.csv gpurun_out/prof_${R4L_TAG:-r4l}/summary.md gpurun_out/prof_${R4L_TAG:-r4l}/bench.log > /dev/null 2>&1
PMC_TAG=pmc_${R4L_TAG:-r4l} PMC_PREC=fp32 BARGS="--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --option face_groups=1" bash tools/runs/pmc.sh || exit 1
SQ_TAG=sq_${R4L_TAG:-r4l} BARGS="--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --option face_groups=1" bash tools/runs/sq.sh > /dev/null || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --precision fp16 --height 2160 --width 3840 --frames-src up2 > $O/c5_fp16.json 2>> $O/c5.err || exit 1
PROF_TAG=prof_${R4L_TAG:-r4l}_c5 PROF_B=64 BARGS="--steps 5 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0 --precision fp16 --height 2160 --width 3840 --frames-src up2" bash tools/runs/prof.sh > /dev/null || exit 1
PMC_TAG=pmc_${R4L_TAG:-r4l}_c5 PMC_PREC=fp16 BARGS="--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --precision fp16 --height 2160 --width 3840 --frames-src up2 --option face_groups=1" bash tools/runs/pmc.sh > /dev/null || exit 1
python tools/prof_summary.py gpurun_out/prof_${R4L_TAG:-r4l}_c5/run_kernel_stats.csv gpurun_out/prof_${R4L_TAG:-r4l}_c5/summary.md gpurun_out/prof_${R4L_TAG:-r4l}_c5/bench.log > /dev/null 2>&1
echo done
