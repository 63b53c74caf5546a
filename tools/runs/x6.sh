#!/bin/bash
# fp32-plan conv layer timings (tools/x6bench): X6_RUNS="label:opts;label:opts" (opts space separated)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${X6_TAG:-x6}
mkdir -p $OUT
IFS=';' read -ra RUNS <<< "${X6_RUNS:-base:}"
for r in "${RUNS[@]}"; do
    name=${r%%:*}; opts=${r#*:}
    echo "== $name ($opts)" | tee -a $OUT/all.txt
    timeout -k 10 ${X6_TIMEOUT:-120} tools/x6bench ${X6_REPS:-20} ${X6_SEL:-all} $opts > $OUT/$name.txt 2>&1 || { cat $OUT/$name.txt; exit 1; }
    cat $OUT/$name.txt >> $OUT/all.txt
done
cat $OUT/all.txt
