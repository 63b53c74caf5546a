#!/bin/bash
# halo tiles with B fragments one column ahead (option x6_halo_pfb): x6bench 3x3 layers, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_TAG=r7j X6_REPS=30 X6_SEL=c2 X6_RUNS="off:x6_halo_pfb=0;on:x6_halo_pfb=1;off2:x6_halo_pfb=0;on2:x6_halo_pfb=1" bash tools/runs/x6.sh
X6_TAG=r7j_ssh X6_REPS=30 X6_SEL=ssh0 X6_RUNS="off:x6_halo_pfb=0;on:x6_halo_pfb=1;off2:x6_halo_pfb=0;on2:x6_halo_pfb=1" bash tools/runs/x6.sh
