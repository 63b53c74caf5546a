#!/bin/bash
# headline A/B of the 1x1 GEMM loop modes (x6_gemm_uni 2 default / 1 / 0), three rounds interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06w
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for cfg in u2 u0 u1; do
    case $cfg in u2) O="";; u0) O="--option x6_gemm_uni=0";; u1) O="--option x6_gemm_uni=1";; esac
    timeout -k 10 300 python bench.py --steps 30 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 $O > $OUT/${cfg}$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${cfg}$r.json'));print('$cfg$r',d['value'],d['ms_per_step'],d['roofline']['frac'])"
  done
done
