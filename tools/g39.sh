# device Huffman coding: jpeg tests, jpeg pipeline bench
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g39
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jpeg.py tests/test_gpu_pipeline.py -p no:cacheprovider > gpurun_out/g39/tests.log 2>&1; rc=$?
tail -15 gpurun_out/g39/tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
timeout -k 10 300 python bench.py --compare "" --no-cpu-baseline --no-timing --steps 10 --option jenc_gpu=$v > gpurun_out/g39/b$v.json 2>gpurun_out/g39/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g39/b$v.json'));print('jenc_gpu=$v',d['value'],d['jpeg_pipeline'])"
done
