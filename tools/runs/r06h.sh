#!/bin/bash
# MFMA + ds_read main-loop microbenchmark (tools/micro/mfma_loop.hip): issue ceilings of the conv body
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06h
timeout -k 10 120 tools/micro/mfma_loop 4000 | tee gpurun_out/r06h/micro.txt
