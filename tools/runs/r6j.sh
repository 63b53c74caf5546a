#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r6j
export TMPDIR=/tmp
timeout -k 10 300 python tools/jpeg_exp.py noise 8 > gpurun_out/r6j/noise.log 2>&1 || { tail -20 gpurun_out/r6j/noise.log; exit 1; }
timeout -k 10 300 python tools/jpeg_exp.py structured 8 > gpurun_out/r6j/struct.log 2>&1 || { tail -20 gpurun_out/r6j/struct.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6j/noise.log gpurun_out/r6j/struct.log
