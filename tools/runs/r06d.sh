#!/bin/bash
# GEMM tiles with pipelined B reads (x6_gemm_pf) and the halo PF + DMA placement together, x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all x6_gemm_pf=1 x6_halo_pf=1 x6_halo_dma=2 > gpurun_out/r06d_check.txt 2>&1 || { cat gpurun_out/r06d_check.txt; exit 1; }
X6_TAG=r06d X6_REPS=20 X6_RUNS="base:;g:x6_gemm_pf=1;all:x6_gemm_pf=1 x6_halo_pf=1 x6_halo_dma=2;base2:;g2:x6_gemm_pf=1;all2:x6_gemm_pf=1 x6_halo_pf=1 x6_halo_dma=2" bash tools/runs/x6.sh > /dev/null || exit 1
awk '{print $1, $NF}' gpurun_out/r06d_check.txt
cd gpurun_out/r06d && paste <(awk '{print $1, $(NF-3)}' base.txt) <(awk '{print $(NF-3)}' g.txt) <(awk '{print $(NF-3)}' all.txt) <(awk '{print $(NF-3)}' base2.txt) <(awk '{print $(NF-3)}' g2.txt) <(awk '{print $(NF-3)}' all2.txt)
