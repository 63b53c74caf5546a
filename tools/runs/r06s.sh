#!/bin/bash
# 1x1 GEMM loop: uniform (x6_gemm_uni 1) vs uniform with one barrier per K tile (2) vs round 5 (0),
# x6bench B = 64, all layers; checks for both new forms
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06s
for m in 1 2; do
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all x6_gemm_uni=$m > gpurun_out/r06s/check$m.txt 2>&1 || { cat gpurun_out/r06s/check$m.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06s/check$m.txt | tr '\n' ' '; echo
done
X6_TAG=r06s X6_REPS=20 X6_RUNS="u1:;u2:x6_gemm_uni=2;u0:x6_gemm_uni=0;u1b:;u2b:x6_gemm_uni=2" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06s && paste <(awk '/us/ {print $1, $(NF-3)}' u1.txt) <(awk '/us/ {print $(NF-3)}' u2.txt) <(awk '/us/ {print $(NF-3)}' u0.txt) <(awk '/us/ {print $(NF-3)}' u1b.txt) <(awk '/us/ {print $(NF-3)}' u2b.txt))
