# plate stream CU mask x release point (fp32 with plates)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g38
for v in 3,0 0,1 0,2 0,4 3,2 3,4 2,2; do
st=${v%,*}; cu=${v#*,}
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --option plate_stage=$st --option plate_cus=$cu > gpurun_out/g38/q$st.$cu.json 2>gpurun_out/g38/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g38/q$st.$cu.json'));print('stage,cus=$v',d['value'],d['ms_per_step'])"
done
