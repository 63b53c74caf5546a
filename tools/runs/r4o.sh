#!/bin/bash
# halo TR tiles + compile-time wait path (no spills): exactness, x6bench, headline A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_gpu_kernels.py -k "halo or tr_tiles or fp32_chain" -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
X6_TAG=x6o X6_RUNS="tr0:x6_halo_tr=0;tr1:x6_halo_tr=1;tr2:x6_halo_tr=2" bash tools/runs/x6.sh > /dev/null || exit 1
B=(python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --no-timing)
for r in 1 2; do for t in 0 1 2; do timeout -k 10 200 "${B[@]}" --option x6_halo_tr=$t > $OUT/t${t}_$r.json 2>> $OUT/bench.err || exit 1; echo "tr=$t $(grep -o '"ms_per_step": [0-9.]*' $OUT/t${t}_$r.json)"; done; done
