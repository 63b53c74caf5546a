set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g7
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jpeg.py > gpurun_out/g7/jpeg.log 2>&1; rc=$?
tail -15 gpurun_out/g7/jpeg.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/g7/bench.json 2> gpurun_out/g7/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g7/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['frac'],d['parity'], d.get('host_pipeline',{}).get('value'), d['ms_breakdown_per_step'], d.get('plate_conv'))"
