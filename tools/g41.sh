# device Huffman + chunked stuffing + packed D2H: jpeg tests, stage split
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g41
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jpeg.py tests/test_gpu_pipeline.py -p no:cacheprovider > gpurun_out/g41/tests.log 2>&1; rc=$?
tail -15 gpurun_out/g41/tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
timeout -k 10 300 python bench.py --compare "" --no-cpu-baseline --no-timing --steps 10 --option jenc_gpu=$v > gpurun_out/g41/b$v.json 2>gpurun_out/g41/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g41/b$v.json'));j=d['jpeg_pipeline'];print('jenc_gpu=$v',j['value'],j['stage_ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g41/prof -o run -- python3 bench.py --compare "" --no-cpu-baseline --no-timing --steps 3 --warmup 1 > gpurun_out/g41/prof.log 2>&1 || exit $?
find gpurun_out/g41/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/g41/stats.csv \;
rm -rf gpurun_out/g41/prof
grep -i "jpeg" gpurun_out/g41/stats.csv | cut -c1-130
