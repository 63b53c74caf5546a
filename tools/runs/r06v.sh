#!/bin/bash
# x6_gemm_uni=2 with the DMA / load order pinned (sched_barrier): repeated checks (the unpinned
# form raced in r06u), timing vs 1 / 0; x6_halo=1 (one-barrier halo, DMA at the top) vs 1b=0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06v
for i in 1 2 3 4 5 6; do
  X6_CHECK=1 timeout -k 10 60 tools/x6bench 2 all > gpurun_out/r06v/c.txt 2>&1 || { cat gpurun_out/r06v/c.txt; exit 1; }
  echo "[$i] $(awk '{print $1, $NF}' gpurun_out/r06v/c.txt | tr '\n' ' ')"
done
X6_CHECK=1 timeout -k 10 60 tools/x6bench 2 all x6_halo=1 > gpurun_out/r06v/c.txt 2>&1 || { cat gpurun_out/r06v/c.txt; exit 1; }
echo "[halo1] $(awk '{print $1, $NF}' gpurun_out/r06v/c.txt | tr '\n' ' ')"
X6_TAG=r06v X6_REPS=20 X6_RUNS="u2:;u1:x6_gemm_uni=1;u0:x6_gemm_uni=0;h1:x6_halo=1;h1o:x6_halo=1 x6_halo_1b=0;u2b:" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06v && paste <(awk '/us/ {print $1, $(NF-3)}' u2.txt) <(awk '/us/ {print $(NF-3)}' u1.txt) <(awk '/us/ {print $(NF-3)}' u0.txt) <(awk '/us/ {print $(NF-3)}' h1.txt) <(awk '/us/ {print $(NF-3)}' h1o.txt) <(awk '/us/ {print $(NF-3)}' u2b.txt))
