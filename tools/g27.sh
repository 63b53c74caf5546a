# EXPERIMENT: which resource bounds the 256x256 pair GEMM (wrong results; timing only)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g27
cd /tmp
for m in 0 4 8 12; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g27/m$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 --option x6_exp=$m > $GRAFT_REPO_ROOT/gpurun_out/g27/m$m.log 2>&1 || exit $?
done
echo ok
