#!/bin/bash
# plate net alone with and without the stride-2 phase halos (option x6_halo_s2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in 0 1; do
  T=r7i/s2_$v
  mkdir -p gpurun_out/$T
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T -o run --output-format csv -- python3 bench.py --faces 0 --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 --no-timing --option x6_halo_s2=$v > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
  K=$(find gpurun_out/$T -name 'run_kernel_trace.csv' | head -1)
  python tools/plate_layers.py "$K" > gpurun_out/$T/plates.txt 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/bench.log
  tail -1 gpurun_out/$T/plates.txt
done
