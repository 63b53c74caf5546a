# plate release at op granularity around face layer3/4 (fp32 with plates)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g43
for i in 1 2; do for v in 31 37 43 47 53; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --option plate_op=$v > gpurun_out/g43/q$v.$i.json 2>gpurun_out/g43/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g43/q$v.$i.json'));print('plate_op=$v',d['value'],d['ms_per_step'])"
done; done
