#!/bin/bash
# fpn.o check errors under x6_halo=1 (seen in r06t): repeat the check per form
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06u
for cfg in "" "x6_halo=1" "x6_halo=1" "x6_halo=1 x6_gemm_uni=1" "x6_halo=1 x6_halo_1b=0" "x6_gemm_uni=1" ""; do
  X6_CHECK=1 timeout -k 10 60 tools/x6bench 2 fpn $cfg > gpurun_out/r06u/c.txt 2>&1 || { cat gpurun_out/r06u/c.txt; exit 1; }
  echo "[$cfg] $(awk '{print $1, $NF}' gpurun_out/r06u/c.txt | tr '\n' ' ')"
done
for cfg in "" "x6_halo=1" "x6_halo=1 x6_gemm_uni=1"; do
  X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all $cfg > gpurun_out/r06u/a.txt 2>&1 || { cat gpurun_out/r06u/a.txt; exit 1; }
  echo "[all $cfg] $(awk '{print $1, $NF}' gpurun_out/r06u/a.txt | tr '\n' ' ')"
done
