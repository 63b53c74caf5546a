#!/bin/bash
# plate stream priority sweep (headline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4z
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
run() { local tag=$1; shift; timeout -k 10 200 "${B[@]}" "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.json)"; }
for r in 1 2; do
  run base_$r
  run hi_$r --option plate_prio=1
  run lo_$r --option plate_prio=2
  run hi_ps4_$r --option plate_prio=1 --option plate_stage=4
  run lo_ps2_$r --option plate_prio=2 --option plate_stage=2
done
