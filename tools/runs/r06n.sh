#!/bin/bash
# full GPU suite + smoke at the current commit, then one headline line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SUITE_TAG=r06n/suite bash tools/runs/suite.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 > gpurun_out/r06n/bench.json 2> gpurun_out/r06n/bench.err || { tail -20 gpurun_out/r06n/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06n/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['per_launch']['frac'],d['blur_roofline']['frac'])"
