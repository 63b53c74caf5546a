# depth-first micro-batching of the early backbone (fp32 pairs), faces only
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g32
for v in 0,2 4,1 8,1 16,1 8,2 16,2 32,1; do
mb=${v%,*}; st=${v#*,}
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 20 --plates 0 --microbatch $mb --microbatch-stage $st > gpurun_out/g32/m$mb.$st.json 2>gpurun_out/g32/m$mb.$st.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/g32/m$mb.$st.json'));print('mb,stage=$v',d['value'],d['ms_per_step'])"
done
