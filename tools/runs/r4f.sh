#!/bin/bash
# mosaic copy-first: exactness tests, blur roofline A/B; vmcnt-form A/B on the fp32 layers
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_capacity.py -k "mosaic or block or layer1 or fused_layer1 or bottleneck" -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for c in 1 0; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --option mosaic_copy=$c > $OUT/copy$c.json 2>> $OUT/bench.err || exit 1; done
X6_TAG=x6f X6_RUNS="imm1:;rt1:x6_dbg=2;imm2:;rt2:x6_dbg=2" bash tools/runs/x6.sh > /dev/null || exit 1
# plate net alone (faces off): per-kernel rocprof stats
mkdir -p gpurun_out/profp_r4f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profp_r4f -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 --faces 0 --plates 1 --no-timing > gpurun_out/profp_r4f/bench.log 2>&1 || exit 1
# block32 per-kernel time in the headline (faces + plates), rocprof stats
mkdir -p gpurun_out/prof_r4f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4f -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 --no-timing > gpurun_out/prof_r4f/bench.log 2>&1 || exit 1
