#!/bin/bash
# plate stream placement test (priorities, CU masks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7k
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_plates.py -k "placement" > gpurun_out/r7k/tests.txt 2>&1 || { tail -40 gpurun_out/r7k/tests.txt; exit 1; }
tail -8 gpurun_out/r7k/tests.txt
