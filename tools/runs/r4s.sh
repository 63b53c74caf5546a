#!/bin/bash
# option sweep under the grouped schedule (headline, no per-launch events)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4s
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
run() { local tag=$1; shift; timeout -k 10 200 "${B[@]}" "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.json)"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "fp32_chain" -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  run base_$r
  run bf32_0_$r --option block_fuse32=0
  run bn256_0_$r --option x6_bn256=0
  run mid_0_$r --option x6_mid=0
  run s256_0_$r --option x6_stream256=0
  run ps2_$r --option plate_stage=2
  run ps4_$r --option plate_stage=4
  run gpw2_$r --option chain_gpw=2
done
