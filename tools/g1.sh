set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g1
export TMPDIR=/tmp
for p in fp32 fp16 bf16; do
  timeout -k 10 300 python bench.py --precision $p --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/g1/bench_$p.json 2> gpurun_out/g1/bench_$p.err || exit $?
  tail -c 600 gpurun_out/g1/bench_$p.json
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g1/prof32 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --precision fp32 --steps 3 --warmup 1 --no-cpu-baseline --no-timing > $GRAFT_REPO_ROOT/gpurun_out/g1/prof32.log 2>&1
echo prof rc=$?
