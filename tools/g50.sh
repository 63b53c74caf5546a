# plate release point re-check after the fused fp32 stem
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g50
for i in 1 2; do for v in 2 3 4; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --option plate_stage=$v > gpurun_out/g50/q$v.$i.json 2>gpurun_out/g50/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g50/q$v.$i.json'));print('plate_stage=$v',d['value'],d['ms_per_step'])"
done; done
