# round-2 closing run: full GPU suite, smoke, default bench line
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/g49
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['jpeg_pipeline']['value'],d['jpeg_pipeline']['stage_ms_per_step'],d['host_pipeline']['value'])"
