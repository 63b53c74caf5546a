set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g3
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_capacity.py tests/test_gpu_configs.py tests/test_gpu_dist.py tests/test_gpu_pipeline.py -s > gpurun_out/g3/new.log 2>&1; rc=$?
tail -15 gpurun_out/g3/new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/g3/bench.json 2> gpurun_out/g3/bench.err || exit $?
cat gpurun_out/g3/bench.json
