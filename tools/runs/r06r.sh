#!/bin/bash
# GEMM two-stage loop on 1x1 convs: uniform loads / DMAs every K tile (x6_gemm_uni 1) vs the round-5
# loop (0), x6bench B = 64, all layers; then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06r
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all > gpurun_out/r06r/check.txt 2>&1 || { cat gpurun_out/r06r/check.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06r/check.txt | tr '\n' ' '; echo
X6_TAG=r06r X6_REPS=20 X6_RUNS="uni:;old:x6_gemm_uni=0;uni2:;old2:x6_gemm_uni=0" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06r && paste <(awk '/us/ {print $1, $(NF-3)}' uni.txt) <(awk '/us/ {print $(NF-3)}' old.txt) <(awk '/us/ {print $(NF-3)}' uni2.txt) <(awk '/us/ {print $(NF-3)}' old2.txt))
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06r/bench.json 2> gpurun_out/r06r/bench.err || { tail -20 gpurun_out/r06r/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r06r/bench.json').read().strip().splitlines()[-1]);print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'],d.get('parity'))"
