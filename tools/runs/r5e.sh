#!/bin/bash
# headline with 1 / 2 / 3 batches in flight (bench.py --inflight), alternating on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_dist.py -x -q --timeout 200 --timeout-method thread -k inflight > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
for r in 1 2; do
  for n in 1 2 3; do
    timeout -k 10 240 "${B[@]}" --inflight $n > $OUT/b_${n}_$r.json 2>> $OUT/err.log || exit 1
    python3 -c "
import json;d=json.loads(open('$OUT/b_${n}_$r.json').read().strip().splitlines()[-1]);print('inflight=$n run $r',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['step']['frac'],d['blur_roofline']['frac'])"
  done
done
