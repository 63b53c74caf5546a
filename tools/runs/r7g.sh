#!/bin/bash
# residual loads ahead of the stores in the 1x1 epilogues: parity, x6bench layers, headline bench x2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7g
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "conv" tests/test_gpu_parity_fp32.py \
  > gpurun_out/r7g/tests.txt 2>&1 || { tail -40 gpurun_out/r7g/tests.txt; exit 1; }
tail -3 gpurun_out/r7g/tests.txt
X6_TAG=r7g X6_REPS=20 X6_RUNS="new:" bash tools/runs/x6.sh
for round in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 > gpurun_out/r7g/ab.json 2> gpurun_out/r7g/ab.err || { tail -5 gpurun_out/r7g/ab.err; exit 1; }
  echo "[new] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7g/ab.json) $(python3 -c "import json;d=json.loads(open('gpurun_out/r7g/ab.json').read().strip().splitlines()[-1]);r=d['roofline'];print('frac',r['frac'],'per_launch',r['per_launch']['frac'],r['per_launch']['avg_launch_ms'])")" | tee -a gpurun_out/r7g/all.txt
done
