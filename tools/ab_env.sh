#!/bin/bash
# A/B of kernel-selection options on one box (vd_set_option through bench.py --option):
#   bash tools/ab_env.sh "chain=1" "chain=0" ...   (several options: "chain=0 conv_n192=0")
# (each config once per round, 3 rounds, 30 timed steps each; prints ms_per_step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2 3; do
  for cfg in "$@"; do
    opts=""; for o in $cfg; do opts="$opts --option $o"; done
    timeout -k 10 200 python bench.py $opts --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
  done
done
