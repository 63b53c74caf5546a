#!/bin/bash
# in-network layer4.0 1x1 convs (l4.0.c1 575 us vs 394 in x6bench): per-layer times under option variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06x
mkdir -p $OUT
for cfg in base bn128 uni0 noplate; do
  case $cfg in base) O="";; bn128) O="--option x6_bn256=0";; uni0) O="--option x6_gemm_uni=0";; noplate) O="--plates 0";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$cfg -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --option face_groups=1 $O > $OUT/$cfg.log 2>&1 || { tail -5 $OUT/$cfg.log; exit 1; }
  K=$(find $OUT/$cfg -name 'run_kernel_trace.csv' | head -1)
  python tools/fp32_layers.py "$K" 64 1 > $OUT/$cfg.layers 2>&1
  echo "[$cfg] $(grep -E '^(l3.1.c1|l3.5.c3|l4.0.c1|l4.0.c2|l4.0.ds|l4.0.c3|l4.1.c1|fpn.o2|total)' $OUT/$cfg.layers | awk '{print $1, $(NF-5)}' | tr '\n' ' ')"
done
