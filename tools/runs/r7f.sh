#!/bin/bash
# stride-2 phase halos: parity (new cases, conv cases, fp32 parity vs oracle), x6bench, headline A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7f
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "halo_s2 or (conv_matches_torch and fp32)" tests/test_gpu_parity_fp32.py \
  > gpurun_out/r7f/tests.txt 2>&1 || { tail -40 gpurun_out/r7f/tests.txt; exit 1; }
tail -3 gpurun_out/r7f/tests.txt
X6_TAG=r7f X6_REPS=20 X6_SEL=.0.c2 X6_RUNS="base:x6_halo_s2=0;s2:x6_halo_s2=1" bash tools/runs/x6.sh
for round in 1 2; do
  for cfg in "x6_halo_s2=0" "x6_halo_s2=1"; do
    timeout -k 10 200 python bench.py --option $cfg --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 > gpurun_out/r7f/ab.json 2> gpurun_out/r7f/ab.err || { tail -5 gpurun_out/r7f/ab.err; exit 1; }
    echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7f/ab.json) $(python3 -c "import json;d=json.loads(open('gpurun_out/r7f/ab.json').read().strip().splitlines()[-1]);r=d['roofline'];print('frac',r['frac'],'per_launch',r['per_launch']['frac'],r['per_launch']['avg_launch_ms'])")" | tee -a gpurun_out/r7f/all.txt
  done
done
