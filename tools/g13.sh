# full GPU suite + smoke + default bench with the fp16-pair fp32 plan as the default
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g13
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/g13/tests.log 2>&1; rc=$?
tail -15 gpurun_out/g13/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g13/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/g13/smoke.log
timeout -k 10 200 python bench.py > gpurun_out/g13/bench.json 2> gpurun_out/g13/bench.err || exit $?
cat gpurun_out/g13/bench.json
