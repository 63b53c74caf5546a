#!/bin/bash
# halo tiles: where the B DMA of step s + 2 is issued (option x6_halo_dma 0 / 1 / 2), x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_TAG=r06b X6_REPS=20 X6_RUNS="base:;d1:x6_halo_dma=1;d2:x6_halo_dma=2;base2:;d2b:x6_halo_dma=2" bash tools/runs/x6.sh > /dev/null || exit 1
cd gpurun_out/r06b && paste <(awk '{print $1, $(NF-3)}' base.txt) <(awk '{print $(NF-3)}' d1.txt) <(awk '{print $(NF-3)}' d2.txt) <(awk '{print $(NF-3)}' base2.txt) <(awk '{print $(NF-3)}' d2b.txt)
