# fp32 fused stem + pool (stem_pool32_kernel): full GPU suite, then faces-only and full A/B
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g45
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/g45/tests.log 2>&1; rc=$?
tail -25 gpurun_out/g45/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 --option stem_pool=$v > gpurun_out/g45/f$v.$i.json 2>gpurun_out/g45/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g45/f$v.$i.json'));print('faces stem_pool=$v',d['value'],d['ms_per_step'])"
done; done
for v in 0 1; do
timeout -k 10 300 python bench.py --compare "fp32_exact" --host-pipeline 0 --steps 20 --option stem_pool=$v > gpurun_out/g45/b$v.json 2>gpurun_out/g45/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g45/b$v.json'));print('full stem_pool=$v',d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity'])"
done
