#!/bin/bash
# mosaic cell kernel timing experiment (wrong outputs for map bits 16/32/64)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5b
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
for m in 1 17 33 65 1 ; do
  timeout -k 10 200 "${B[@]}" --option mosaic_map=$m --option mosaic_cells=16 > $OUT/b_$m.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json;d=json.loads(open('$OUT/b_$m.json').read().strip().splitlines()[-1]);b=d['blur_roofline'];print('map=$m',d['ms_per_step'],b['avg_launch_ms'],b['family']['avg_ms_per_step'])"
done
