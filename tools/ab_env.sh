#!/bin/bash
# A/B of environment switches on one box: bash tools/ab_env.sh "VD_X=1" "VD_X=0" ...
# (each config once per round, 3 rounds, 30 timed steps each; prints ms_per_step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2 3; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
  done
done
