#!/bin/bash
# SQ counters of the headline bench (two rocprofv3 --pmc passes, 8 SQ counters each),
# per kernel name: launches and the mean of each counter per launch. SQ_TAG names the
# output, BARGS the bench arguments, SQ_FILTER a regex of kernel names to print.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
T=gpurun_out/${SQ_TAG:-sq}
BARGS=${BARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing"}
mkdir -p $T
eval timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $T/a -o run --output-format csv -- python3 bench.py $BARGS > $T/a.log 2>&1 || { tail -5 $T/a.log; exit 1; }
eval timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -d $T/b -o run --output-format csv -- python3 bench.py $BARGS > $T/b.log 2>&1 || { tail -5 $T/b.log; exit 1; }
python - <<PY
import csv, glob, re
from collections import defaultdict
flt = re.compile("${SQ_FILTER:-conv|bottleneck|stem}")
per = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for d in ("$T/a", "$T/b"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if not flt.search(k): continue
        per[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, d)].add(r["Dispatch_Id"])
out = []
for k in sorted(per):
    na = max(len(n[(k, "$T/a")]), 1); nb = max(len(n[(k, "$T/b")]), 1)
    c = {x: v / (na if x in ("SQ_WAVES","SQ_INSTS_VALU","SQ_INSTS_MFMA","SQ_INSTS_LDS","SQ_INSTS_VMEM","SQ_INSTS_SALU","SQ_WAVE_CYCLES","SQ_BUSY_CYCLES") else nb) for x, v in per[k].items()}
    mf = max(c.get("SQ_INSTS_MFMA", 0), 1)
    wc = max(c.get("SQ_WAVE_CYCLES", 0), 1)
    out.append(f"{k[:52]:52s} n={na:3d} valu/mfma={c.get('SQ_INSTS_VALU',0)/mf:5.2f} lds/mfma={c.get('SQ_INSTS_LDS',0)/mf:5.2f} vmem/mfma={c.get('SQ_INSTS_VMEM',0)/mf:5.2f} "
               f"wait_any/wave={c.get('SQ_WAIT_ANY',0)/wc:.3f} wait_inst/wave={c.get('SQ_WAIT_INST_ANY',0)/wc:.3f} wait_lds/wave={c.get('SQ_WAIT_INST_LDS',0)/wc:.3f} "
               f"act_valu/wave={c.get('SQ_ACTIVE_INST_VALU',0)/wc:.3f} act_mfma/wave={c.get('SQ_ACTIVE_INST_MFMA',0)/wc:.3f} act_lds/wave={c.get('SQ_ACTIVE_INST_LDS',0)/wc:.3f} "
               f"act_vmem/wave={c.get('SQ_ACTIVE_INST_VMEM',0)/wc:.3f} bank_conf={c.get('SQ_LDS_BANK_CONFLICT',0):.3g}")
open("$T/summary.txt", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
