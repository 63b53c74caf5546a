#!/bin/bash
# Full GPU suite (oracle parity first, conftest.py orders it) + smoke, as the driver runs them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${SUITE_TAG:-suite}
mkdir -p $OUT
export TMPDIR=/tmp VD_PARITY_OUT=$OUT/parity
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests -p no:cacheprovider ${PYTEST_EXTRA:-} > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
