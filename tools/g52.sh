# 256-channel dual (layer1.0 conv3 + downsample): parity, faces-only A/B against the committed build
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g52
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "dual or fp32" -p no:cacheprovider > gpurun_out/g52/tests.log 2>&1; rc=$?
tail -3 gpurun_out/g52/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 1 0; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 --option x6_stream256=$((v*2)) > gpurun_out/g52/f$v.$i.json 2>gpurun_out/g52/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g52/f$v.$i.json'));print('faces s256=$((v*2))',d['value'],d['ms_per_step'])"
done; done
