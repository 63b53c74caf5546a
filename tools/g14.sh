# per-layer fp32 (pair) profiles, faces only: default tile selection vs big tile forced for N<=64
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g14
export TMPDIR=/tmp
A="--steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare '' --host-pipeline 0 --plates 0"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g14/p0 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 > $GRAFT_REPO_ROOT/gpurun_out/g14/p0.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g14/p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 --option x6_small_k=0 --option x6_small_tiles=0 > $GRAFT_REPO_ROOT/gpurun_out/g14/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g14/p2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 --plates 0 --option x6_small_k=100000 --option x6_stream=0 > $GRAFT_REPO_ROOT/gpurun_out/g14/p2.log 2>&1 || exit $?
echo ok
