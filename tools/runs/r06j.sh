#!/bin/bash
# kernel trace of the headline steps (no instrumented pass): per-stream timeline of a step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06j
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06j/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 --no-timing > gpurun_out/r06j/trace.log 2>&1 || { tail -5 gpurun_out/r06j/trace.log; exit 1; }
python tools/step_timeline.py gpurun_out/r06j/trace | tee gpurun_out/r06j/timeline.txt
