# decode-ahead GPU codec path of batch_process_images
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g48
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_jpeg.py -p no:cacheprovider > gpurun_out/g48/tests.log 2>&1; rc=$?
tail -3 gpurun_out/g48/tests.log
exit $rc
