#!/bin/bash
# layer1 block HBM fetch per launch (FETCH_SIZE, gfx950 x2 correction): pipelined vs one-group kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6k
mkdir -p $OUT
for pp in 1 0; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/f$pp -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --plates 0 --option block32_pipe=$pp > $OUT/f$pp.log 2>&1 || { tail -5 $OUT/f$pp.log; exit 1; }
  D=$(dirname $(find $OUT/f$pp -name 'run_kernel_trace.csv' | head -1))
  python3 - "$D" $pp <<'PY'
import csv, os, sys
d, pp = sys.argv[1], sys.argv[2]
tr = {r["Dispatch_Id"]: r["Kernel_Name"] for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))}
agg = {}
for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
    if r["Counter_Name"] != "FETCH_SIZE": continue
    k = tr.get(r["Dispatch_Id"], "?")
    if "bottleneck32" not in k: continue
    k = k.split("(")[0].replace("(anonymous namespace)::", "")[-60:]
    agg.setdefault(k, []).append(2 * float(r["Counter_Value"]) * 1024 / 1e9)
for k, v in agg.items():
    print(f"pipe={pp} {k}: {len(v)} launches, fetch {sum(v)/len(v):.3f} GB per launch (x = 1.678 GB)")
PY
done
