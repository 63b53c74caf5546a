#!/bin/bash
# JPEG pipeline (structured / noise frames, overlapped stages): kernel time by stage
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06o
for k in structured noise; do
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06o/$k -o run --output-format csv -- python3 tools/jpeg_exp.py $k 8 true > gpurun_out/r06o/$k.log 2>&1 || { tail -5 gpurun_out/r06o/$k.log; exit 1; }
grep frames/s gpurun_out/r06o/$k.log; grep "alone" gpurun_out/r06o/$k.log
python tools/jpeg_kernels.py gpurun_out/r06o/$k
done
