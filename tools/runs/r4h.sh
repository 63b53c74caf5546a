#!/bin/bash
# face net as two half batches on two streams (option face_halves): exactness, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
# (tests green: gpurun_out/r4h/tests.log of the first call)


B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0)
for i in 1 2; do
  for hv in 1 0; do timeout -k 10 200 "${B[@]}" --option face_halves=$hv > $OUT/h${hv}_$i.json 2>> $OUT/bench.err || exit 1; done
done
for hv in 1 0; do timeout -k 10 200 "${B[@]}" --plates 0 --option face_halves=$hv > $OUT/faces_h$hv.json 2>> $OUT/bench.err || exit 1; done
