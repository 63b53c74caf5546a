# stream-K (one block per range, two segments): parity, A/B, traces
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g35
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "stream_k" -p no:cacheprovider > gpurun_out/g35/tests.log 2>&1; rc=$?
tail -2 gpurun_out/g35/tests.log
[ $rc -eq 0 ] || exit $rc
for v in 0,16 1,16 1,8 1,30; do
sk=${v%,*}; mn=${v#*,}
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 --option x6_sk=$sk --option x6_sk_min=$mn > gpurun_out/g35/p$sk.$mn.json 2>gpurun_out/g35/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g35/p$sk.$mn.json'));print('sk,min=$v',d['value'],d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g35/prof1 -o run -- python3 bench.py --faces 1 --plates 0 --compare "" --no-cpu-baseline --host-pipeline 0 --steps 3 --warmup 1 --no-timing --option x6_sk=1 --option x6_sk_min=8 > gpurun_out/g35/prof1.log 2>&1 || exit $?
find gpurun_out/g35/prof1 -name '*kernel_trace.csv' -exec cp {} gpurun_out/g35/trace1.csv \;
rm -rf gpurun_out/g35/prof1
