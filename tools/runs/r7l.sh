#!/bin/bash
# default switches re-checked at the round's last kernel commit (ms/step, two rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7l
for round in 1 2; do
  for cfg in "" "plate_stage=2" "plate_stage=4" "chain=1" "face_groups=3" "block32_pipe=0"; do
    opts=""; for o in $cfg; do opts="$opts --option $o"; done
    timeout -k 10 200 python bench.py $opts --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing > gpurun_out/r7l/ab.json 2> gpurun_out/r7l/ab.err || { tail -5 gpurun_out/r7l/ab.err; exit 1; }
    echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7l/ab.json)" | tee -a gpurun_out/r7l/all.txt
  done
done
