#!/bin/bash
# fused mosaic band height (option mosaic_rows 16 / 24 / 32, 0 = auto): exactness, then the blur
# roofline of C2 (720p bf16 B=32), C3 (1080p fp32 B=64) and C5 (4K fp16 B=64)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_kernels.py -k "mosaic_fused" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
C2="--height 720 --width 1280 --batch 32 --precision bf16 --frames-src up2"
C5="--height 2160 --width 3840 --batch 64 --precision fp16 --frames-src up2 --steps 10 --warmup 2"
RS="${ROWS_SET:-16 8 16g 8g}"
for r in $RS; do
  G=0; case $r in *g) G=1; r=${r%g};; esac
  for cfg in C2 C5 C3; do
    case $cfg in C2) A=$C2;; C5) A=$C5;; C3) A="";; esac
    timeout -k 10 300 python bench.py $A --compare "" --no-cpu-baseline --host-pipeline 0 --option mosaic_rows=$r --option mosaic_gather=$G > $OUT/${cfg}_$r$G.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${cfg}_$r$G.json'));b=d['blur_roofline'];print('$cfg rows=$r gather=$G',d['value'],d['ms_per_step'],'blur',b['frac'],b['avg_launch_ms'])"
  done
done
