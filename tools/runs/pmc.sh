#!/bin/bash
# HBM traffic per launch (face convs, mosaic_out_kernel): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes of the same bench command, then tools/pmc_traffic.py
# (KiB counters, gfx950 FETCH_SIZE correction). PMC_TAG names the output, BARGS the bench
# arguments, PMC_PREC the precision label.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
T=${PMC_TAG:-pmc}
BARGS=${BARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing"}
mkdir -p gpurun_out/$T
eval timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/fetch -o run --output-format csv -- python3 bench.py $BARGS > gpurun_out/$T/fetch.log 2>&1 || { tail -5 gpurun_out/$T/fetch.log; exit 1; }
eval timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$T/write -o run --output-format csv -- python3 bench.py $BARGS > gpurun_out/$T/write.log 2>&1 || { tail -5 gpurun_out/$T/write.log; exit 1; }
F=$(dirname $(find gpurun_out/$T/fetch -name 'run_kernel_trace.csv' | head -1))
W=$(dirname $(find gpurun_out/$T/write -name 'run_kernel_trace.csv' | head -1))
python tools/pmc_traffic.py $F $W gpurun_out/$T/traffic.json ${PMC_PREC:-fp32} | tail -12
