#!/bin/bash
# RetinaFace heads on the streaming form (option x6_stream_heads): heads parity, rocprof of the heads, headline x2 each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r7r
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r7r/p$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --plates 0 --option face_groups=1 --option x6_stream_heads=$v > gpurun_out/r7r/p$v.log 2>&1 || { tail -5 gpurun_out/r7r/p$v.log; exit 1; }
  echo "== heads $v"; grep -h "conv_x6_kernel<128, 32\|conv1x1_x6_kernel<8, 2," $(find gpurun_out/r7r/p$v -name 'run_kernel_stats.csv') | cut -c1-160
done
for round in 1 2; do for v in 0 1; do
  timeout -k 10 200 python bench.py --option x6_stream_heads=$v --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing > gpurun_out/r7r/ab.json 2> gpurun_out/r7r/ab.err || { tail -5 gpurun_out/r7r/ab.err; exit 1; }
  echo "[heads=$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7r/ab.json)"
done; done
