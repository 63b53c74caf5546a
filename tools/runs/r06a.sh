#!/bin/bash
# round 6 first box: the changed GPU tests, a headline bench line and x6bench per-layer baseline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_lib_abi.py tests/test_gpu_shard.py tests/test_gpu_plates.py "tests/test_gpu_kernels.py::test_mosaic_output_forms_match_oracle" \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --host-pipeline 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d.get('cpu_baseline',{}).get('value'),d.get('cpu_baseline',{}).get('per_frame'))"
X6_TAG=r06a/x6 X6_REPS=20 X6_RUNS="base:" bash tools/runs/x6.sh > /dev/null || exit 1
cat $OUT/x6/base.txt
