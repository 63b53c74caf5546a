#!/bin/bash
# vmcnt-form A/B on the fp32 layers, then the headline's rocprof kernel stats and PMC traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
X6_TAG=x6e X6_RUNS="imm1:;rt1:x6_dbg=2;imm2:;rt2:x6_dbg=2" bash tools/runs/x6.sh > /dev/null || exit 1
PROF_TAG=prof_r4e bash tools/runs/prof.sh || exit 1
PMC_TAG=pmc_r4e bash tools/runs/pmc.sh || exit 1
