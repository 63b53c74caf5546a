# 192-wide pair tile: conv / e2e parity, faces-only layer profile, default bench
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g16
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_e2e.py -k "fp32" -p no:cacheprovider > gpurun_out/g16/tests.log 2>&1; rc=$?
tail -5 gpurun_out/g16/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g16/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 > $GRAFT_REPO_ROOT/gpurun_out/g16/p.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --compare "" --host-pipeline 0 --no-cpu-baseline > gpurun_out/g16/bench.json 2> gpurun_out/g16/bench.err || exit $?
cat gpurun_out/g16/bench.json
