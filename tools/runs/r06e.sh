#!/bin/bash
# new conv schedule defaults: bit-identity + conv / parity tests, then headline A/B (round-5 schedule vs new)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_e2e.py tests/test_gpu_parity_fp32.py "tests/test_gpu_kernels.py" -k "fp32 or halo or conv" \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="python bench.py --steps 20 --warmup 3 --compare '' --host-pipeline 0 --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --host-pipeline 0 --no-cpu-baseline --option x6_halo_pf=0 --option x6_gemm_pf=0 --option x6_halo_dma=0 > $OUT/old$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --host-pipeline 0 --no-cpu-baseline > $OUT/new$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
for f in old1 new1 old2 new2; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline'].get('per_launch'))"; done
