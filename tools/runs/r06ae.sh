#!/bin/bash
# stream-level defaults re-checked on the final kernels: face_groups 2 (default) / 1 / 3, plate_stage 3 (default) / 2,
# two interleaved rounds of headline lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06ae
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in base g1 g3 ps2; do
    case $cfg in base) O="";; g1) O="--option face_groups=1";; g3) O="--option face_groups=3";; ps2) O="--option plate_stage=2";; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 $O > $OUT/${cfg}$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${cfg}$r.json'));print('$cfg$r',d['value'],d['ms_per_step'],d['roofline']['frac'])"
  done
done
