#!/bin/bash
# fp32 oracle parity at every config size (tests/test_gpu_parity_fp32.py), records under gpurun_out/parity
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/parity
export TMPDIR=/tmp VD_PARITY_OUT=gpurun_out/parity
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m parity tests -p no:cacheprovider > gpurun_out/parity/tests.log 2>&1; rc=$?
tail -5 gpurun_out/parity/tests.log
exit $rc
