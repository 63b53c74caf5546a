# x6 VALU trims (32-bit offsets, select-only tap advance, fma-mix split, 2 waves/EU bound): parity + bench + layer profile
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g24
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_plates.py -k "fp32" -p no:cacheprovider > gpurun_out/g24/tests.log 2>&1; rc=$?
tail -4 gpurun_out/g24/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 > gpurun_out/g24/faces.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/g24/faces.json'));print('faces',d['value'],d['ms_per_step'])"
timeout -k 10 200 python bench.py --compare "fp32_x6" --host-pipeline 0 > gpurun_out/g24/bench.json 2> gpurun_out/g24/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g24/bench.json'));print('full',d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g24/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 > $GRAFT_REPO_ROOT/gpurun_out/g24/p.log 2>&1 || exit $?
