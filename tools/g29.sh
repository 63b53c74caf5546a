# plate branch release point (plate_stage) x plate stream priority, fp32 with plates
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g29
export TMPDIR=/tmp
for i in 1 2; do for v in 3,0 3,1 3,-1 2,1 2,-1 0,-1 0,1; do
st=${v%,*}; pr=${v#*,}
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --option plate_stage=$st --option plate_prio=$pr > gpurun_out/g29/q$st.$pr.$i.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/g29/q$st.$pr.$i.json'));print('stage,prio=$v',d['value'],d['ms_per_step'])"
done; done
