#!/bin/bash
# plates-only kernel trace (bench --faces 0): per-launch view of the plate net; then the block PMC fetch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6l
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --faces 0 --steps 5 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
K=$(find $OUT/prof -name 'run_kernel_trace.csv' | head -1)
python tools/plate_layers.py "$K" > $OUT/plate_layers.txt 2>&1 || true
cat $OUT/plate_layers.txt
tools/runs/r6k.sh
