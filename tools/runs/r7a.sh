#!/bin/bash
# 1x1 GEMM layers: full launch vs main loop only (x6_dbg=1 skips the epilogue), x6bench B=64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_TAG=r7a X6_REPS=20 X6_RUNS="base:;noepi:x6_dbg=1" bash tools/runs/x6.sh
