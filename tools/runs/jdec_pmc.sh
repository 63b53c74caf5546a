#!/bin/bash
# SQ counters of the device JPEG decode kernels (tools/jdec_prof.py, 2 decodes), two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${JDEC_TAG:-jdecpmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $OUT/a -o run --output-format csv -- python3 tools/jdec_prof.py noise 1 > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/b -o run --output-format csv -- python3 tools/jdec_prof.py noise 1 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
python - <<PY
import csv, glob
from collections import defaultdict
for d in ("$OUT/a", "$OUT/b"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    per = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if "jdec" not in k and "jpeg" not in k: continue
        per[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k in per:
        print(k, len(n[k]), " ".join(f"{c}={v/len(n[k]):.3g}" for c, v in sorted(per[k].items())))
PY
