# decode-ahead jpeg pipeline + zero-copy decode input: jpeg/pipeline tests, bench
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g47
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jpeg.py tests/test_gpu_pipeline.py -p no:cacheprovider > gpurun_out/g47/tests.log 2>&1; rc=$?
tail -3 gpurun_out/g47/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --compare "" --no-cpu-baseline --no-timing --steps 10 > gpurun_out/g47/b.json 2>gpurun_out/g47/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g47/b.json'));j=d['jpeg_pipeline'];print(d['value'],j['value'],j['stage_ms_per_step'])"
