#!/bin/bash
# A/B of kernel-selection options on the headline bench (one process per arm, fixed order,
# repeated): AB_ARMS="name1:--option a=1 name2:" ; optional PYTEST_K runs GPU tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${AB_TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "${PYTEST_K:-}" ]; then
    timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider -k "$PYTEST_K" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
    tail -2 $OUT/tests.log
fi
BARGS=${BARGS:-"--steps 10 --warmup 3 --compare '' --host-pipeline 0 --no-cpu-baseline"}
for rep in $(seq ${AB_REPS:-2}); do
  for arm in ${AB_ARMS}; do
    name=${arm%%:*}; opts=${arm#*:}; opts=${opts//,/ }
    eval timeout -k 10 300 python bench.py $BARGS $opts > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { tail -20 $OUT/$name.$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/$name.$rep.json')); print('$name', $rep, d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('ms_breakdown_per_step',{}).get('conv'))"
  done
done
