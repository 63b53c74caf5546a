# stream-K default: full GPU suite, then full bench A/B (faces + plates)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g36
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/g36/tests.log 2>&1; rc=$?
tail -3 gpurun_out/g36/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --option x6_sk=$v > gpurun_out/g36/p$v.$i.json 2>gpurun_out/g36/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g36/p$v.$i.json'));print('sk=$v',d['value'],d['ms_per_step'])"
done; done
