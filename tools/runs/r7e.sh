#!/bin/bash
# plate branch stream placement under face groups: priority high / low, CU masks (ms_per_step, 2 rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7e
for round in 1 2; do
  for cfg in "" "plate_prio=2" "plate_prio=1" "plate_prio=3 plate_cus=32" "plate_prio=3 plate_cus=64" "plate_prio=3 plate_cus=128"; do
    opts=""; for o in $cfg; do opts="$opts --option $o"; done
    timeout -k 10 200 python bench.py $opts --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing > gpurun_out/r7e/ab.json 2> gpurun_out/r7e/ab.err || { tail -5 gpurun_out/r7e/ab.err; exit 1; }
    echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7e/ab.json)" | tee -a gpurun_out/r7e/all.txt
  done
done
