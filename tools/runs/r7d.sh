#!/bin/bash
# conv1x1_tr2p_kernel with the per-group LDS max merge: parity tests, x6bench with / without max slots
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7d
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "tr2" tests/test_gpu_e2e.py::test_heads_fp32_x6_tr2_bit_identical \
  > gpurun_out/r7d/tests.txt 2>&1 || { tail -40 gpurun_out/r7d/tests.txt; exit 1; }
tail -3 gpurun_out/r7d/tests.txt
X6_TAG=r7d X6_REPS=20 X6_SEL=. X6_RUNS="base:;p1:x6_tr2p=1" bash tools/runs/x6.sh
X6_NOYMAX=1 X6_TAG=r7d_noy X6_REPS=20 X6_SEL=. X6_RUNS="base:;p1:x6_tr2p=1" bash tools/runs/x6.sh
