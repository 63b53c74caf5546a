#!/bin/bash
# mosaic cell kernel: batched gathers, workgroups-per-frame sweep (mosaicbench + headline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5a
mkdir -p $OUT
export TMPDIR=/tmp
for c in 4 8 16 32; do
  timeout -k 10 120 python tools/mosaicbench.py --option mosaic_cells=$c > $OUT/mb_$c.json 2>> $OUT/err.log || exit 1
  echo "cells=$c $(cat $OUT/mb_$c.json)"
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread -k mosaic > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
for c in 8 16 32; do
  timeout -k 10 200 "${B[@]}" --option mosaic_cells=$c > $OUT/b_$c.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json;d=json.loads(open('$OUT/b_$c.json').read().strip().splitlines()[-1]);print('bench cells=$c',d['ms_per_step'],d['blur_roofline']['frac'],d['blur_roofline']['family'])"
done
