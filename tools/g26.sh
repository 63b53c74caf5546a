# exact-canvas stem (one A plane): bit-identity + fp32 parity, jpeg tests, faces-only layer profile, bench
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g26
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_gpu_jpeg.py tests/test_gpu_pipeline.py -k "fp32 or jpeg or encode or decode or codec" -p no:cacheprovider > gpurun_out/g26/tests.log 2>&1; rc=$?
tail -4 gpurun_out/g26/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g26/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 > $GRAFT_REPO_ROOT/gpurun_out/g26/p.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --compare "" --no-cpu-baseline > gpurun_out/g26/bench.json 2> gpurun_out/g26/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g26/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['jpeg_pipeline']['value'],d['host_pipeline']['value'])"
