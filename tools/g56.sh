# final safety run: full GPU suite + smoke on the committed tree
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g56
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/g56/tests.log 2>&1; rc=$?
tail -2 gpurun_out/g56/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/g56/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/g56/smoke.log
