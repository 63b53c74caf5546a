# plate co-scheduling: face branch at high stream priority vs not; faces-only reference
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g19
A="--compare '' --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30"
for i in 1 2; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 > gpurun_out/g19/base$i.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --option face_hi_prio=1 > gpurun_out/g19/hi$i.json 2>/dev/null || exit $?
done
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 > gpurun_out/g19/faces.json 2>/dev/null || exit $?
for f in gpurun_out/g19/*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
