#!/bin/bash
# Cout-128 halo layers as two 64-wide N tiles (x6_halo_n64): SSH level-0/1 conv5X5_2 + conv7X7_2, layer2 conv2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 ssh x6_halo_n64=4096 > gpurun_out/r06q_check.txt 2>&1 || { cat gpurun_out/r06q_check.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06q_check.txt | tr '\n' ' '; echo
for sel in ssh0.c52 ssh1.c52 ssh0.c73 l2.1.c2; do
X6_TAG=r06q_$sel X6_SEL=$sel X6_REPS=20 X6_RUNS="base:;n64:x6_halo_n64=4096;base2:;n64b:x6_halo_n64=4096" bash tools/runs/x6.sh > /dev/null || exit 1
for f in base n64 base2 n64b; do echo "$sel $f $(awk '/us/ {print $(NF-3)}' gpurun_out/r06q_$sel/$f.txt | head -1)"; done
done
