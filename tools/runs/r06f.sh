#!/bin/bash
# effective shader clock per kernel (GRBM_GUI_ACTIVE pass) on the headline bench command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06f
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r06f/clk -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --compare "" --host-pipeline 0 --no-timing > gpurun_out/r06f/clk.log 2>&1 || { tail -5 gpurun_out/r06f/clk.log; exit 1; }
python tools/clock_pmc.py gpurun_out/r06f/clk 100 | tee gpurun_out/r06f/clock.txt
