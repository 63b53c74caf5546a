#!/bin/bash
# streaming 1x1 (l3.x.c3, l2.1.c3, l4.1.c3, l2.0.c1): epilogue cost (x6_dbg=1), the RL form (residual loaded
# beside the MFMAs, x6_stream_rl=1), the TR GEMM tile instead (x6_gemm1x1=2); x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 c3 x6_stream_rl=1 > gpurun_out/r06l_check.txt 2>&1 || { cat gpurun_out/r06l_check.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06l_check.txt
for sel in l3.1.c3 l2.1.c3 l4.1.c3 l2.0.c1; do
X6_TAG=r06l_$sel X6_SEL=$sel X6_REPS=20 X6_RUNS="base:;rl:x6_stream_rl=1;noepi:x6_dbg=1;tr:x6_gemm1x1=2;base2:;rl2:x6_stream_rl=1" bash tools/runs/x6.sh > /dev/null || exit 1
for f in base rl noepi tr base2 rl2; do echo "$sel $f $(awk '/us/ {print $(NF-3)}' gpurun_out/r06l_$sel/$f.txt | head -1)"; done
done
