#!/bin/bash
# stride-2 halo layers: timing-only skips (x6_dbg bits 2-5 -> hdbg: 4 no B DMA, 8 no halo reload,
# 32 no main-loop barriers; WRONG results), x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06aa
for sel in l2.0.c2 l3.0.c2 l4.0.c2 l2.1.c2 l3.1.c2; do
  line="$sel"
  for d in 0 4 8 32 44; do
    timeout -k 10 60 tools/x6bench 20 $sel x6_dbg=$d > gpurun_out/r06aa/o.txt 2>&1 || { cat gpurun_out/r06aa/o.txt; exit 1; }
    line="$line d$d=$(awk '/us/ && $1=="'$sel'" {print $(NF-3)}' gpurun_out/r06aa/o.txt)"
  done
  echo "$line"
done
