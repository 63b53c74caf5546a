# plates-only kernel trace (plate net per-layer view) + plate/pipeline GPU tests
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g30
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g30/prof -o run -- python3 bench.py --faces 0 --compare "" --no-cpu-baseline --host-pipeline 0 --steps 5 --warmup 2 --no-timing > gpurun_out/g30/bench.log 2>&1 || exit $?
find gpurun_out/g30/prof -name '*kernel_trace.csv' -exec cp {} gpurun_out/g30/trace.csv \;
find gpurun_out/g30/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/g30/stats.csv \;
rm -rf gpurun_out/g30/prof
