set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g8
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g8/profp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --faces 0 > $GRAFT_REPO_ROOT/gpurun_out/g8/profp.log 2>&1
echo rc=$?
