set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g5
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g5/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $GRAFT_REPO_ROOT/gpurun_out/g5/prof.log 2>&1
echo rc=$?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g5/prof_np -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 > $GRAFT_REPO_ROOT/gpurun_out/g5/prof_np.log 2>&1
echo rc=$?
