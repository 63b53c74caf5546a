# full GPU suite + smoke + default bench (all round-2 changes)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g25
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/g25/tests.log 2>&1; rc=$?
tail -6 gpurun_out/g25/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g25/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/g25/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/g25/bench.json 2> gpurun_out/g25/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g25/bench.json'));print(d['value'],d['ms_per_step'],d['roofline'],d['parity'],d.get('jpeg_pipeline',{}).get('value'),d['host_pipeline']['value'])"
