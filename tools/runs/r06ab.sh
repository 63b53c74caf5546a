#!/bin/bash
# stride-2 halo layers: B DMA placement (x6_halo_dma 0 after the barrier / 1 after the MFMAs / 2 pieces
# between MFMA groups, default) and B-read pipelining (x6_halo_pf), x6bench B = 64, two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06ab
for pass in 1 2; do
for sel in l2.0.c2 l3.0.c2 l4.0.c2; do
  line="$sel"
  for o in "x6_halo_dma=2" "x6_halo_dma=0" "x6_halo_dma=1" "x6_halo_pf=0"; do
    timeout -k 10 60 tools/x6bench 20 $sel $o > gpurun_out/r06ab/o.txt 2>&1 || { cat gpurun_out/r06ab/o.txt; exit 1; }
    line="$line $o:$(awk '/us/ && $1=="'$sel'" {print $(NF-3)}' gpurun_out/r06ab/o.txt)"
  done
  echo "$line"
done
done
