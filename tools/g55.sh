# fused fp32 stem: LDS swizzle for stage B's two pool pixels per 16 lanes
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g55
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "fp32" -p no:cacheprovider > gpurun_out/g55/tests.log 2>&1; rc=$?
tail -2 gpurun_out/g55/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --steps 30 --plates 0 > gpurun_out/g55/f.$i.json 2>gpurun_out/g55/err.txt || exit $?
python -c "import json;d=json.load(open('gpurun_out/g55/f.$i.json'));print('faces',d['value'],d['ms_per_step'])"
done
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/g55/sq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 > $GRAFT_REPO_ROOT/gpurun_out/g55/sq.log 2>&1 || exit $?
grep -h "stem_pool32" $(find $GRAFT_REPO_ROOT/gpurun_out/g55/sq -name '*counter_collection.csv') | cut -c1-20 > /dev/null
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g55/sq/**/*counter_collection.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "stem_pool32" in r["Kernel_Name"]:
        print(r["Counter_Name"], r["Counter_Value"])
PY
