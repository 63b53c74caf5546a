#!/bin/bash
# C5 (4K up2, fp16 plan) option sweep: frames/s and the conv-family fraction
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r4y
mkdir -p $OUT
export TMPDIR=/tmp
B=(python bench.py --steps 8 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --precision fp16 --height 2160 --width 3840 --frames-src up2)
run() { local tag=$1; shift; timeout -k 10 200 "${B[@]}" "$@" > $OUT/$tag.json 2>> $OUT/bench.err || exit 1; python3 -c "
import json,sys;d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['step']['frac'])"; }
run base
run kmin256 --option conv_big_kmin=256
run big50 --option conv_big=50
run big200 --option conv_big=200
run small256 --option conv_small=256
run small1024 --option conv_small=1024
run ntt8 --option stream_ntt=8
run n192_0 --option conv_n192=0
run side1 --option ssh_side=1
