# JPEG encode leg: GPU parity vs Pillow bytes
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g18
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jpeg.py tests/test_gpu_kernels.py -k "encode or decode or case9 or case10" -p no:cacheprovider > gpurun_out/g18/tests.log 2>&1; rc=$?
tail -15 gpurun_out/g18/tests.log
exit $rc
