# profiles for the round-2 headline (fp32 split): kernel-trace stats, then the two PMC passes
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g10
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g10/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 > $GRAFT_REPO_ROOT/gpurun_out/g10/prof.log 2>&1 || exit $?
echo prof ok
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/g10/pmc_fetch -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $GRAFT_REPO_ROOT/gpurun_out/g10/pmc_fetch.log 2>&1 || exit $?
echo fetch ok
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/g10/pmc_write -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $GRAFT_REPO_ROOT/gpurun_out/g10/pmc_write.log 2>&1 || exit $?
echo write ok
