#!/bin/bash
# Device JPEG decode alone (tools/jdec_prof.py): option sweep, then a rocprof kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${JDEC_TAG:-jdec}
mkdir -p $OUT
export TMPDIR=/tmp
for arm in ${JDEC_ARMS:-"noise"}; do
  args=${arm//,/ }
  timeout -k 10 300 python tools/jdec_prof.py $args >> $OUT/sweep.log 2>&1 || { tail -20 $OUT/sweep.log; exit 1; }
done
cat $OUT/sweep.log
if [ -n "${JDEC_PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/jdec_prof.py $JDEC_PROF > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  S=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1)
  python -c "
import csv
for x in csv.DictReader(open('$S')):
    print(f\"{x['Name'][:70]:70s} {x['Calls']:>5} {float(x['TotalDurationNs'])/1e6:9.2f} ms {float(x['AverageNs'])/1e3:9.1f} us\")"
fi
