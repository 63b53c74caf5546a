#!/bin/bash
# fp32 layer2 chain (chain32.hip): exactness vs the two-launch plan, fp32 parity, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "fp32_chain or fused_layer1 or fp32_parity or oracle" -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
for c in 1 0 1; do timeout -k 10 200 "${B[@]}" --option chain=$c > $OUT/chain$c.json 2>> $OUT/bench.err || exit 1; echo "chain=$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/chain$c.json)"; done
mkdir -p gpurun_out/prof_r4m
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4m -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 > gpurun_out/prof_r4m/bench.log 2>&1 || exit 1
python tools/fp32_layers.py gpurun_out/prof_r4m/run_kernel_trace.csv > gpurun_out/prof_r4m/layers.txt 2>&1
