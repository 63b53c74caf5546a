# jpeg pipeline stage split, device vs host entropy encode
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g40
for v in 1 0; do
timeout -k 10 300 python bench.py --compare "" --no-cpu-baseline --no-timing --steps 10 --option jenc_gpu=$v > gpurun_out/g40/b$v.json 2>gpurun_out/g40/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g40/b$v.json'));j=d['jpeg_pipeline'];print('jenc_gpu=$v',j['value'],j['stage_ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g40/prof -o run -- python3 bench.py --compare "" --no-cpu-baseline --no-timing --steps 3 --warmup 1 > gpurun_out/g40/prof.log 2>&1 || exit $?
find gpurun_out/g40/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/g40/stats.csv \;
rm -rf gpurun_out/g40/prof
grep -i "jpeg" gpurun_out/g40/stats.csv | cut -c1-160
