#!/bin/bash
# halo tiles: where the time goes -- timing-only skips (x6_dbg bits: 4 no B DMA, 8 no halo reload,
# 32 no barriers, 1 no epilogue), x6bench B = 64, fpn.m1 / l3.1.c2 / ssh0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for sel in m1 l3.1.c2 ssh0; do
X6_TAG=r06g_$sel X6_SEL=$sel X6_REPS=20 X6_RUNS="base:;noepi:x6_dbg=1;nodma:x6_dbg=4;nohalo:x6_dbg=8;nodmahalo:x6_dbg=12;nobar:x6_dbg=32;none:x6_dbg=45;base2:" bash tools/runs/x6.sh > /dev/null || exit 1
for f in base noepi nodma nohalo nodmahalo nobar none base2; do echo "$sel $f $(awk '/us/ {print $(NF-3)}' gpurun_out/r06g_$sel/$f.txt | head -1)"; done
done
