#!/bin/bash
# TR 1x1 layers on the one-barrier loop: full launch vs main loop only (timing-only x6_dbg=1 skips the
# epilogue: WRONG results), x6bench B = 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06af
for sel in l2.0.ds l3.0.c1 l3.0.ds l3.1.c1 l4.0.c1 l4.0.ds l4.1.c1 l4.1.c3 l4.0.c3 fpn.o1 fpn.o2; do
  line="$sel"
  for d in 0 1 0 1; do
    timeout -k 10 60 tools/x6bench 20 $sel x6_dbg=$d > gpurun_out/r06af/o.txt 2>&1 || { cat gpurun_out/r06af/o.txt; exit 1; }
    line="$line d$d=$(awk '/us/ && $1=="'$sel'" {print $(NF-3)}' gpurun_out/r06af/o.txt)"
  done
  echo "$line"
done
