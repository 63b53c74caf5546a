#!/bin/bash
# block32 stage-1 depth: bit-identity tests, then headline A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4x
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
run() { local tag=$1; shift; timeout -k 10 200 "${B[@]}" "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.json)"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "block32_depth or fused_layer1" -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing --option face_groups=1 --option block32_xd=4 > $OUT/prof.log 2>&1 || exit 1
grep bottleneck32 $(find $OUT/prof -name 'run_kernel_stats.csv') | cut -c1-160
for r in 1 2; do
  run base_$r
  run xd3_$r --option block32_xd=3
  run xd4_$r --option block32_xd=4
done
