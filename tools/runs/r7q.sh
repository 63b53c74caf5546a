#!/bin/bash
# headline repeatability on one box: 5 runs of the timed steps (20 steps each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7q
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 > gpurun_out/r7q/b$i.json 2> gpurun_out/r7q/b$i.err || { tail -5 gpurun_out/r7q/b$i.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/r7q/b$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('run $i', d['value'], d['ms_per_step'], r['frac'], r['per_launch']['frac'], d['blur_roofline']['frac'])" | tee -a gpurun_out/r7q/all.txt
done
