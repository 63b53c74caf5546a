#!/bin/bash
# TR register epilogue: residual / BN rows of pair jp + 1 before pair jp's stores (x6_tr_epi 1) vs the
# round-5 row-by-row form (0), x6bench B = 64, all layers (the halo tiles share the epilogue)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all > gpurun_out/r06m_check.txt 2>&1 || { cat gpurun_out/r06m_check.txt; exit 1; }
X6_TAG=r06m X6_REPS=20 X6_RUNS="new:;old:x6_tr_epi=0;new2:;old2:x6_tr_epi=0" bash tools/runs/x6.sh > /dev/null || exit 1
awk '{print $1, $NF}' gpurun_out/r06m_check.txt | tr '\n' ' '; echo
cd gpurun_out/r06m && paste <(awk '/us/ {print $1, $(NF-3)}' new.txt) <(awk '/us/ {print $(NF-3)}' old.txt) <(awk '/us/ {print $(NF-3)}' new2.txt) <(awk '/us/ {print $(NF-3)}' old2.txt)
