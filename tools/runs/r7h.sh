#!/bin/bash
# uneven face frame groups (option face_group_split): headline ms/step, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r7h
for round in 1 2; do
  for cfg in "face_group_split=0" "face_group_split=40" "face_group_split=45" "face_group_split=55" "face_group_split=60"; do
    timeout -k 10 200 python bench.py --option $cfg --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing > gpurun_out/r7h/ab.json 2> gpurun_out/r7h/ab.err || { tail -5 gpurun_out/r7h/ab.err; exit 1; }
    echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7h/ab.json)" | tee -a gpurun_out/r7h/all.txt
  done
done
