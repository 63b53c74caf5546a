#!/bin/bash
# mosaic cell kernel with separable candidate masks: mosaic tests, then the headline's blur family
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_golden.py tests/test_gpu_capacity.py tests/test_gpu_configs.py tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread -k "mosaic" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
for r in 1 2; do
  for c in 32 16; do
    timeout -k 10 240 "${B[@]}" --option mosaic_cells=$c > $OUT/b_${c}_$r.json 2>> $OUT/err.log || exit 1
    python3 -c "
import json;d=json.loads(open('$OUT/b_${c}_$r.json').read().strip().splitlines()[-1]);b=d['blur_roofline'];print('cells=$c run $r',d['ms_per_step'],b['frac'],b['family'])"
  done
done
