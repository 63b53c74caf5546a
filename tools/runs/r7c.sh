#!/bin/bash
# conv1x1_tr2p_kernel: parity tests, then x6bench 1x1 layers with x6_tr2p = 0 / 1 / 2 (+ no epilogue)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7c
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "tr2" tests/test_gpu_e2e.py::test_heads_fp32_x6_tr2_bit_identical \
  > gpurun_out/r7c/tests.txt 2>&1 || { tail -40 gpurun_out/r7c/tests.txt; exit 1; }
tail -3 gpurun_out/r7c/tests.txt
X6_TAG=r7c X6_REPS=20 X6_SEL=. X6_RUNS="base:;p1:x6_tr2p=1;p2:x6_tr2p=2;p2min1:x6_tr2p=2 x6_tr2p_min=1;p2noepi:x6_tr2p=2 x6_dbg=1" bash tools/runs/x6.sh
