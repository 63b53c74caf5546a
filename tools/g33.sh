# stream-K: conv parity, fp32 suites, then faces-only A/B
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g33
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "stream_k or (conv_matches_torch and fp32) or split_error" -p no:cacheprovider > gpurun_out/g33/tests.log 2>&1; rc=$?
tail -5 gpurun_out/g33/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 --option x6_sk=$v > gpurun_out/g33/p$v.$i.json 2>gpurun_out/g33/p$v.$i.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g33/p$v.$i.json'));print('sk=$v',d['value'],d['ms_per_step'])"
done; done
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --steps 20 > gpurun_out/g33/full.json 2>gpurun_out/g33/full.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g33/full.json'));print('full',d['value'],d['ms_per_step'],d.get('parity'))"
