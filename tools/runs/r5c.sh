#!/bin/bash
# plates-only kernel trace (per-launch plate-net view) + headline stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/plates -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --faces 0 > $OUT/plates.json 2>> $OUT/err.log || exit 1
f=$(find $OUT/plates -name '*kernel_trace.csv' | head -1)
python tools/plate_layers.py "$f" > $OUT/plate_layers.txt || exit 1
cat $OUT/plate_layers.txt
