# plate_stage parity
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g31
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_plates.py -k "release or paired or faces_and_plates" -p no:cacheprovider > gpurun_out/g31/tests.log 2>&1; rc=$?
tail -3 gpurun_out/g31/tests.log
exit $rc
