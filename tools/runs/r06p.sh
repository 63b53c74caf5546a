#!/bin/bash
# JPEG pipeline: device entropy decode (default) vs the host Huffman threads (jdec_gpu=0), structured / noise
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06p
for k in structured noise; do
  for o in jdec_gpu=1 jdec_gpu=0; do
    timeout -k 10 300 python3 tools/jpeg_exp.py $k 8 true $o > gpurun_out/r06p/${k}_$o.log 2>&1 || { tail -5 gpurun_out/r06p/${k}_$o.log; exit 1; }
    echo "$k $o $(grep frames/s gpurun_out/r06p/${k}_$o.log)"
  done
done
nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
