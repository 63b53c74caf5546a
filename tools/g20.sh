# plate net alone (fp32 pair plan): kernel trace
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g20
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g20/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --faces 0 > $GRAFT_REPO_ROOT/gpurun_out/g20/p.log 2>&1 || exit $?
echo ok
