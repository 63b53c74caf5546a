#!/bin/bash
# halo tiles on two B stages (x6_halo=1 forces them; at 1080p the stride-8 256-wide layers take them):
# one barrier per step (x6_halo_1b 1) vs two (0), and the three-stage default; x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06t
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all x6_halo=1 > gpurun_out/r06t/check.txt 2>&1 || { cat gpurun_out/r06t/check.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06t/check.txt | tr '\n' ' '; echo
X6_TAG=r06t X6_REPS=20 X6_RUNS="n3:;b1:x6_halo=1;b2:x6_halo=1 x6_halo_1b=0;b1d0:x6_halo=1 x6_halo_dma=0;b1r:x6_halo=1;b2r:x6_halo=1 x6_halo_1b=0" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06t && paste <(awk '/us/ {print $1, $(NF-3)}' n3.txt) <(awk '/us/ {print $(NF-3)}' b1.txt) <(awk '/us/ {print $(NF-3)}' b2.txt) <(awk '/us/ {print $(NF-3)}' b1d0.txt) <(awk '/us/ {print $(NF-3)}' b1r.txt) <(awk '/us/ {print $(NF-3)}' b2r.txt))
