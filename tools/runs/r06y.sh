#!/bin/bash
# 1x1 Cout >= 512 layers on the 128 x 128 TR tile (two workgroups per CU) for K <= x6_mid_wide, x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06y
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all x6_mid_wide=1024 > gpurun_out/r06y/check.txt 2>&1 || { cat gpurun_out/r06y/check.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06y/check.txt | tr '\n' ' '; echo
X6_TAG=r06y X6_REPS=20 X6_RUNS="base:;w512:x6_mid_wide=512;w1024:x6_mid_wide=1024;base2:;w2048:x6_mid_wide=2048" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06y && paste <(awk '/us/ {print $1, $(NF-3)}' base.txt) <(awk '/us/ {print $(NF-3)}' w512.txt) <(awk '/us/ {print $(NF-3)}' w1024.txt) <(awk '/us/ {print $(NF-3)}' base2.txt) <(awk '/us/ {print $(NF-3)}' w2048.txt))
