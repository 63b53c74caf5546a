#!/bin/bash
# hardware queues per process (GPU_MAX_HW_QUEUES 4 = HIP default, 8, 16) x batches in flight
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5f
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
for r in 1 2; do
  for q in 4 8 16; do
    for n in 1 2; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 240 "${B[@]}" --inflight $n > $OUT/b_${q}_${n}_$r.json 2>> $OUT/err.log || exit 1
      python3 -c "
import json;d=json.loads(open('$OUT/b_${q}_${n}_$r.json').read().strip().splitlines()[-1]);print('queues=$q inflight=$n run $r',d['value'],d['ms_per_step'])"
    done
  done
done
