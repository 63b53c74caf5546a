# stream-K threshold sweep (faces only) + kernel traces sk on/off
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g34
for v in 0,16 1,16 1,24 1,40 1,1000; do
sk=${v%,*}; mn=${v#*,}
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 --option x6_sk=$sk --option x6_sk_min=$mn > gpurun_out/g34/p$sk.$mn.json 2>gpurun_out/g34/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g34/p$sk.$mn.json'));print('sk,min=$v',d['value'],d['ms_per_step'])"
done
for sk in 0 1; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g34/prof$sk -o run -- python3 bench.py --faces 1 --plates 0 --compare "" --no-cpu-baseline --host-pipeline 0 --steps 3 --warmup 1 --no-timing --option x6_sk=$sk --option x6_sk_min=16 > gpurun_out/g34/prof$sk.log 2>&1 || exit $?
find gpurun_out/g34/prof$sk -name '*kernel_trace.csv' -exec cp {} gpurun_out/g34/trace$sk.csv \;
rm -rf gpurun_out/g34/prof$sk
done
