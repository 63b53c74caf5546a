#!/bin/bash
# stride-2 halo tiles after inlining s2_tap / s2_last (they were real calls, each entry a
# vmcnt(0) lgkmcnt(0) drain): checks + x6bench B = 64 all layers twice; headline line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06z
X6_CHECK=1 timeout -k 10 120 tools/x6bench 2 all > gpurun_out/r06z/check.txt 2>&1 || { cat gpurun_out/r06z/check.txt; exit 1; }
awk '{print $1, $NF}' gpurun_out/r06z/check.txt | tr '\n' ' '; echo
X6_TAG=r06z X6_REPS=20 X6_RUNS="a:;b:" bash tools/runs/x6.sh > /dev/null || exit 1
(cd gpurun_out/r06z && paste <(awk '/us/ {print $1, $(NF-3)}' a.txt) <(awk '/us/ {print $(NF-3)}' b.txt))
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 > gpurun_out/r06z/bench$r.json 2> gpurun_out/r06z/bench.err || { tail -20 gpurun_out/r06z/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06z/bench$r.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['per_launch']['frac'])"
done
