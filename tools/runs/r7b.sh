#!/bin/bash
# conv1x1_tr2_kernel: parity tests, then x6bench TR layers with x6_tr2 = 0 / 1 / 2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7b
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "tr2 or tr_tiles" tests/test_gpu_e2e.py::test_heads_fp32_x6_tr2_bit_identical \
  > gpurun_out/r7b/tests.txt 2>&1 || { tail -40 gpurun_out/r7b/tests.txt; exit 1; }
tail -3 gpurun_out/r7b/tests.txt
X6_TAG=r7b X6_REPS=20 X6_RUNS="base:;tr2:x6_tr2=1;tr2s:x6_tr2=2;tr2noepi:x6_tr2=2 x6_dbg=1" bash tools/runs/x6.sh
