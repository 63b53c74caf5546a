# fp32 space-to-depth stem: letterbox/e2e/plates/config tests, faces-only + full A/B
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g44
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_configs.py tests/test_gpu_plates.py -p no:cacheprovider > gpurun_out/g44/tests.log 2>&1; rc=$?
tail -15 gpurun_out/g44/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 --option stem_s2d32=$v > gpurun_out/g44/f$v.$i.json 2>gpurun_out/g44/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g44/f$v.$i.json'));print('faces s2d32=$v',d['value'],d['ms_per_step'])"
done; done
for v in 0 1; do
timeout -k 10 300 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --steps 20 --option stem_s2d32=$v > gpurun_out/g44/b$v.json 2>gpurun_out/g44/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g44/b$v.json'));print('full s2d32=$v',d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity']['fp32_vs_oracle'])"
done
