#!/bin/bash
# halo tiles: pipelined B-fragment reads (option x6_halo_pf) x DMA placement (x6_halo_dma), x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 c2 x6_halo_pf=1 > gpurun_out/r06c_check.txt 2>&1 || { cat gpurun_out/r06c_check.txt; exit 1; }
X6_TAG=r06c X6_REPS=20 X6_RUNS="base:;pf:x6_halo_pf=1;pfd1:x6_halo_pf=1 x6_halo_dma=1;pfd2:x6_halo_pf=1 x6_halo_dma=2;base2:;pf2:x6_halo_pf=1" bash tools/runs/x6.sh > /dev/null || exit 1
cat gpurun_out/r06c_check.txt | tail -8
cd gpurun_out/r06c && paste <(awk '{print $1, $(NF-3)}' base.txt) <(awk '{print $(NF-3)}' pf.txt) <(awk '{print $(NF-3)}' pfd1.txt) <(awk '{print $(NF-3)}' pfd2.txt) <(awk '{print $(NF-3)}' base2.txt) <(awk '{print $(NF-3)}' pf2.txt)
