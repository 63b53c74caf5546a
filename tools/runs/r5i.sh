#!/bin/bash
# plate branch release point with face groups (plate_stage 1..4), headline, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5i
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
for r in 1 2; do
  for ps in 3 1 2 4; do
    timeout -k 10 240 "${B[@]}" --option plate_stage=$ps > $OUT/b_${ps}_$r.json 2>> $OUT/err.log || exit 1
    python3 -c "
import json;d=json.loads(open('$OUT/b_${ps}_$r.json').read().strip().splitlines()[-1]);print('plate_stage=$ps run $r',d['value'],d['ms_per_step'])"
  done
done
