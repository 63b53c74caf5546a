set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "fp32" > gpurun_out/g4/conv.log 2>&1; rc=$?
tail -15 gpurun_out/g4/conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_gpu_dist.py tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_capacity.py -s > gpurun_out/g4/e2e.log 2>&1; rc=$?
tail -15 gpurun_out/g4/e2e.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/g4/bench.json 2> gpurun_out/g4/bench.err || exit $?
cat gpurun_out/g4/bench.json
