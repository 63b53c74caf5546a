set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g9
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "fp32" > gpurun_out/g9/conv.log 2>&1; rc=$?
tail -3 gpurun_out/g9/conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --compare "" --host-pipeline 0 --plates 0 > gpurun_out/g9/bench_np.json 2> gpurun_out/g9/bench_np.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g9/bench_np.json'));print('noplates',d['value'],d['ms_per_step'],d['roofline']['achieved'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --compare "" --host-pipeline 0 > gpurun_out/g9/bench.json 2> gpurun_out/g9/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g9/bench.json'));print('plates',d['value'],d['ms_per_step'],d['roofline']['achieved'])"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g9/prof_np -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 > $GRAFT_REPO_ROOT/gpurun_out/g9/prof_np.log 2>&1
echo prof rc=$?
