#!/bin/bash
# plate branch scheduling: Detect levels early + face mosaic before the plate join (options
# plate_detect_early / mosaic_early) -- identity test, headline A/B (two rounds), timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_plates.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for cfg in old new ps1 ps2; do
    case $cfg in old) O="--option plate_detect_early=0 --option mosaic_early=0";; new) O="";;
                 ps1) O="--option plate_stage=1";; ps2) O="--option plate_stage=2";; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 $O > $OUT/${cfg}$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${cfg}$r.json'));print('$cfg$r',d['value'],d['ms_per_step'],d['roofline']['frac'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 --no-timing > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python tools/step_timeline.py $OUT/trace | tee $OUT/timeline.txt | grep -v tail
