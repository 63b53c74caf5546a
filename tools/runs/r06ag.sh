#!/bin/bash
# streaming 1x1: RL form (one register set, refills per k-step, frame range one group ahead through a
# buffer load) also for the layers without a residual (x6_stream_rl 2) vs residual-only (1, default);
# x6bench B = 64 check + A/B, then headline lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06ag
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all x6_stream_rl=2 > gpurun_out/r06ag/check.txt 2>&1 || { cat gpurun_out/r06ag/check.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06ag/check.txt | tr '\n' ' '; echo
X6_TAG=r06ag X6_REPS=20 X6_RUNS="rl1:;rl2:x6_stream_rl=2;rl1b:;rl2b:x6_stream_rl=2" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06ag && paste <(awk '/us/ {print $1, $(NF-3)}' rl1.txt) <(awk '/us/ {print $(NF-3)}' rl2.txt) <(awk '/us/ {print $(NF-3)}' rl1b.txt) <(awk '/us/ {print $(NF-3)}' rl2b.txt))
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in rl1 rl2; do
    case $cfg in rl1) O="";; rl2) O="--option x6_stream_rl=2";; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 $O > gpurun_out/r06ag/${cfg}$r.json 2>> gpurun_out/r06ag/err.log || { tail -20 gpurun_out/r06ag/err.log; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ag/${cfg}$r.json'));print('$cfg$r',d['value'],d['ms_per_step'],d['roofline']['frac'])"
  done
done
