# GPU session: new tests first (capacity, configs, dist), then the rest, smoke, bench
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_capacity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -s > gpurun_out/g2/new.log 2>&1; rc=$?
tail -5 gpurun_out/g2/new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_capacity.py --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_dist.py > gpurun_out/g2/rest.log 2>&1; rc=$?
tail -5 gpurun_out/g2/rest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g2/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/g2/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/g2/bench.json 2> gpurun_out/g2/bench.err || exit $?
cat gpurun_out/g2/bench.json
