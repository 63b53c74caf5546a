# x6 wave priority A/B (faces only, fp32)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g23
for i in 1 2; do
for v in 0 1; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 --option x6_prio=$v > gpurun_out/g23/p$v.$i.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/g23/p$v.$i.json'));print('prio=$v',d['value'],d['ms_per_step'])"
done; done
