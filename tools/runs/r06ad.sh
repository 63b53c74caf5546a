#!/bin/bash
# round-5/6 GEMM defaults re-checked on the one-barrier 1x1 loop: x6_mid=0 (Cout-128 1x1 on 256x128),
# x6_gemm_pf=0, x6_adepth=4; x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06ad
X6_TAG=r06ad X6_REPS=20 X6_RUNS="base:;mid0:x6_mid=0;pf0:x6_gemm_pf=0;ad4:x6_adepth=4;base2:" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06ad && paste <(awk '/us/ {print $1, $(NF-3)}' base.txt) <(awk '/us/ {print $(NF-3)}' mid0.txt) <(awk '/us/ {print $(NF-3)}' pf0.txt) <(awk '/us/ {print $(NF-3)}' ad4.txt) <(awk '/us/ {print $(NF-3)}' base2.txt))
