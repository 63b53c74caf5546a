#!/bin/bash
# fp32 headline: option spot-check at the last commit (two rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5j
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
run() { local tag=$1; shift; timeout -k 10 200 "${B[@]}" "$@" > $OUT/$tag.json 2>> $OUT/err.log || exit 1; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.json)"; }
for r in 1 2; do
  run base_$r
  run cells16_$r --option mosaic_cells=16
  run adepth4_$r --option x6_adepth=4
  run mid0_$r --option x6_mid=0
  run s256_1_$r --option x6_stream256=1
  run chain1_$r --option chain=1
  run halotr1_$r --option x6_halo_tr=1
done
