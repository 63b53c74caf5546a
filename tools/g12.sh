# fp16-pair fp32 plan (f32_split=2): conv / e2e / plate parity, bench vs the bf16 triple, per-layer profile
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g12
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_plates.py -k "pair or split or fp32" -p no:cacheprovider > gpurun_out/g12/tests.log 2>&1; rc=$?
tail -25 gpurun_out/g12/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --precision fp32_pair --compare fp32 --host-pipeline 0 > gpurun_out/g12/bench.json 2> gpurun_out/g12/bench.err || exit $?
cat gpurun_out/g12/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g12/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --precision fp32_pair --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $GRAFT_REPO_ROOT/gpurun_out/g12/prof.log 2>&1 || exit $?
echo prof ok
